"""Probe of the HIP runtime's bookkeeping for page-locked host ranges.

Queries only, apart from guarded copies: hipHostRegister / hipHostUnregister of ranges that share
pages with each other and with unregistered neighbours, then hipPointerGetAttributes and
hsa_amd_pointer_info on every interesting address (first / last byte of each range, the shared
page, the bytes of a range's first / last page outside it) after each step.  A pageable
device-to-host copy into a page is made only when both queries call that page unknown to the
runtime, and its data are checked.

    python scripts/hostreg_probe.py [--torch]   # --torch: import torch first (its bundled HIP runtime,
                                                # the one the pytest process binds); else /opt/rocm's
Output: one JSON object per line (stdout).
"""
import ctypes as C
import json
import mmap
import sys

USE_TORCH = "--torch" in sys.argv
if USE_TORCH:
    import torch  # noqa: F401  (its libamdhip64 / libhsa-runtime64 are then the process's)

    torch.cuda.init()

hip = C.CDLL("libamdhip64.so.7")
hsa = C.CDLL("libhsa-runtime64.so.1")
PAGE = mmap.PAGESIZE


class HipAttr(C.Structure):
    _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p),
                ("hostPointer", C.c_void_p), ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]


class HsaInfo(C.Structure):
    _fields_ = [("size", C.c_uint32), ("type", C.c_int), ("agentBaseAddress", C.c_void_p),
                ("hostBaseAddress", C.c_void_p), ("sizeInBytes", C.c_size_t), ("userData", C.c_void_p),
                ("agentOwner", C.c_uint64), ("global_flags", C.c_uint32), ("registered", C.c_bool)]


hip.hipPointerGetAttributes.argtypes = [C.POINTER(HipAttr), C.c_void_p]
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
hip.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
hip.hipGetErrorString.restype = C.c_char_p
hip.hipGetLastError.restype = C.c_int
hsa.hsa_amd_pointer_info.argtypes = [C.c_void_p, C.POINTER(HsaInfo), C.c_void_p, C.c_void_p, C.c_void_p]
HSA_TYPES = {0: "unknown", 1: "hsa", 2: "locked", 3: "graphics", 4: "ipc", 5: "reserved", 6: "vmem"}


def out(**kw):
    print(json.dumps(kw), flush=True)


def err(e):
    return hip.hipGetErrorString(e).decode()


def query(label, addr, base):
    a = HipAttr()
    e = hip.hipPointerGetAttributes(C.byref(a), C.c_void_p(addr))
    hip.hipGetLastError()  # a failed query sets the sticky-free last error; clear it
    h = HsaInfo()
    h.size = C.sizeof(HsaInfo)
    s = hsa.hsa_amd_pointer_info(C.c_void_p(addr), C.byref(h), None, None, None)
    rec = {"q": label, "off": addr - base, "hip": err(e), "hip_type": a.type if e == 0 else None,
           "hip_dev": hex(a.devicePointer or 0) if e == 0 else None,
           "hip_host": (a.hostPointer or 0) - base if e == 0 and a.hostPointer else None,
           "hsa_status": s, "hsa_type": HSA_TYPES.get(h.type, h.type)}
    if h.type:
        rec.update(hsa_host_off=(h.hostBaseAddress or 0) - base, hsa_agent=hex(h.agentBaseAddress or 0),
                   hsa_size=h.sizeInBytes, hsa_registered=bool(h.registered))
    return rec


def known(rec):
    """page-locked in HIP's view (hipPointerGetAttributes answers hipSuccess for pageable memory too, with type 0 =
    hipMemoryTypeUnregistered) or known to ROCr"""
    return (rec["hip"] == "no error" and rec["hip_type"] not in (None, 0)) or rec["hsa_type"] != "unknown"


def scan(step, base, ranges, extra=()):
    """Query the first / last byte of every range, the bytes just outside it, and its pages' ends."""
    pts = []
    for name, (a, n) in ranges.items():
        pts += [(f"{name}.first", a), (f"{name}.last", a + n - 1), (f"{name}.before", a - 8),
                (f"{name}.after", a + n + 8), (f"{name}.page0", a - a % PAGE),
                (f"{name}.pageN", ((a + n - 1) | (PAGE - 1)))]
    pts += list(extra)
    res = []
    for label, addr in pts:
        r = query(label, addr, base)
        r["step"] = step
        out(**r)
        res.append(r)
    return res


def guarded_copy(step, dev, base, addr, nbytes):
    """Pageable D2H copy into [addr, addr + nbytes) only if every page of it is unknown to the runtime."""
    pages = range(addr - addr % PAGE, addr + nbytes, PAGE)
    stale = [p - base for p in pages if known(query("copy-check", p, base))]
    if stale:
        out(step=step, copy="skipped", reason="pages still known to the runtime", pages=stale)
        return
    e = hip.hipMemcpy(C.c_void_p(addr), dev, C.c_size_t(nbytes), 2)
    got = C.string_at(addr, nbytes)
    out(step=step, copy=err(e), data_ok=got == bytes([0x5A]) * nbytes, off=addr - base, nbytes=nbytes)


def main():
    out(runtime="torch-bundled" if USE_TORCH else "/opt/rocm", page=PAGE)
    arena = mmap.mmap(-1, 64 * PAGE)
    base = C.addressof(C.c_char.from_buffer(arena))
    dev = C.c_void_p()
    assert hip.hipMalloc(C.byref(dev), C.c_size_t(16 * PAGE)) == 0
    assert hip.hipMemset(dev, 0x5A, C.c_size_t(16 * PAGE)) == 0
    C.memset(base, 0x11, 64 * PAGE)

    # S1: two registrations sharing one page, each also sharing its outer pages with unregistered bytes
    A = (base + 128, 5 * PAGE + 1000)
    B = (A[0] + A[1], 2 * PAGE + 64)
    R = {"A": A, "B": B}
    for nm, (a, n) in R.items():
        out(step="S1", reg=nm, rc=err(hip.hipHostRegister(C.c_void_p(a), C.c_size_t(n), 1)))
    scan("S1 both registered", base, R)
    out(step="S1", unreg="A", rc=err(hip.hipHostUnregister(C.c_void_p(A[0]))))
    scan("S1 A unregistered", base, R)
    out(step="S1", unreg="B", rc=err(hip.hipHostUnregister(C.c_void_p(B[0]))))
    scan("S1 both unregistered", base, R)
    guarded_copy("S1 copy into A's first page", dev, base, base + 8, 512)
    guarded_copy("S1 copy into the shared page", dev, base, A[0] + A[1] - 256, 512)

    # S2: register, unregister, then a different range over the same pages (a later heap object)
    Cr = (base + 16 * PAGE + 256, 3 * PAGE)
    D = (base + 16 * PAGE + 64, 4 * PAGE)
    out(step="S2", reg="C", rc=err(hip.hipHostRegister(C.c_void_p(Cr[0]), C.c_size_t(Cr[1]), 1)))
    out(step="S2", unreg="C", rc=err(hip.hipHostUnregister(C.c_void_p(Cr[0]))))
    out(step="S2", reg="D", rc=err(hip.hipHostRegister(C.c_void_p(D[0]), C.c_size_t(D[1]), 1)))
    scan("S2 D registered over C's pages", base, {"C": Cr, "D": D})
    out(step="S2", unreg="D", rc=err(hip.hipHostUnregister(C.c_void_p(D[0]))))
    scan("S2 D unregistered", base, {"C": Cr, "D": D})
    guarded_copy("S2 copy into C/D pages", dev, base, base + 16 * PAGE + 8, 2048)

    # S3: page-exact registration (what the library registers after the fix): whole pages only
    E = (base + 32 * PAGE, 4 * PAGE)
    out(step="S3", reg="E", rc=err(hip.hipHostRegister(C.c_void_p(E[0]), C.c_size_t(E[1]), 1)))
    scan("S3 E registered", base, {"E": E})
    out(step="S3", unreg="E", rc=err(hip.hipHostUnregister(C.c_void_p(E[0]))))
    scan("S3 E unregistered", base, {"E": E})
    guarded_copy("S3 copy into E", dev, base, E[0] + 100, 4096)

    # S4: a registration whose range lies inside the first page of another, nested ranges
    F = (base + 40 * PAGE + 100, 2 * PAGE)
    G = (base + 40 * PAGE + 100 + 2 * PAGE, 200)  # starts in F's last page, ends in it
    for nm, (a, n) in (("F", F), ("G", G)):
        out(step="S4", reg=nm, rc=err(hip.hipHostRegister(C.c_void_p(a), C.c_size_t(n), 1)))
    scan("S4 F,G registered", base, {"F": F, "G": G})
    out(step="S4", unreg="F", rc=err(hip.hipHostUnregister(C.c_void_p(F[0]))))
    scan("S4 F unregistered", base, {"F": F, "G": G})
    out(step="S4", unreg="G", rc=err(hip.hipHostUnregister(C.c_void_p(G[0]))))
    scan("S4 G unregistered", base, {"F": F, "G": G})
    guarded_copy("S4 copy into F/G pages", dev, base, base + 40 * PAGE + 8, 3 * PAGE)

    # S5: a large pageable D2H copy (the runtime may pin the destination on the fly and keep it),
    # then the destination unmapped and a new mapping made (often at the same address)
    big_n = 256 << 20
    dbig = C.c_void_p()
    assert hip.hipMalloc(C.byref(dbig), C.c_size_t(big_n)) == 0
    assert hip.hipMemset(dbig, 0x5A, C.c_size_t(big_n)) == 0
    m1 = mmap.mmap(-1, big_n)
    b1 = C.addressof(C.c_char.from_buffer(m1))
    e = hip.hipMemcpy(C.c_void_p(b1), dbig, C.c_size_t(big_n), 2)
    out(step="S5", copy_big=err(e), data_ok=C.string_at(b1 + big_n - 64, 64) == bytes([0x5A]) * 64)
    for lab, off in (("first", 0), ("mid", big_n // 2), ("last", big_n - 1)):
        r = query(f"S5 after big copy {lab}", b1 + off, b1)
        out(**r)
    m1.close()
    for lab, off in (("first", 0), ("mid", big_n // 2)):
        r = query(f"S5 after unmap {lab}", b1 + off, b1)
        out(**r)
    m2 = mmap.mmap(-1, big_n)
    b2 = C.addressof(C.c_char.from_buffer(m2))
    out(step="S5", remap_same_address=b2 == b1)
    for lab, off in (("first", 0), ("mid", big_n // 2)):
        r = query(f"S5 after remap {lab}", b2 + off, b2)
        out(**r)
    guarded_copy("S5 small copy into the new mapping", dev, b2, b2 + 4096, 8192)
    out(done=True)


if __name__ == "__main__":
    main()
