"""wavespec_amd -- MI355X-native spectrum hot path of WaveSpecZZ.

The product is libmtbridge.so (HIP for gfx950, C ABI of include/mtbridge.h);
this package is its Python host mirror.  See DESIGN.md.
"""
from . import bridge, cycle_cache, indicator, sharding, synth  # noqa: F401

__all__ = ["bridge", "cycle_cache", "indicator", "sharding", "synth"]
