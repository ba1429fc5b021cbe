#!/bin/bash
# The one GPU-box runner: executes the given steps in order, each under its own time limit, and stops
# at the first step that fails (a fault, abort, time limit or test failure ends the call there).
# Everything lands under gpurun_out/<tag>/; copy what is to be judged into profiles/.
#
#   gpurun -- bash scripts/gpu_run.sh <tag> <step> [<step> ...]
#
# steps:
#   tests[=<pytest args>]    pytest -m gpu (default: the whole GPU suite; args comma-separated, '+' = space
#                            inside one, e.g. tests=tests/test_gpu_parity.py,-k,kalman+or+jump), log tests.log
#   smoke                    __graft_entry__.smoke()
#   bench=<cfg>[,<args>]     python bench.py --config <cfg> --steps 100 --warmup 20 --no-cpu-baseline <args>
#                            (args comma-separated), line bench_<cfg>.json
#   benchc=<cfg>[,<args>]    the same with the CPU baseline (1 core + the job's cores) in the line
#   default                  python bench.py (the driver's default line, CPU baseline included)
#   prof=<cfg>[,<algo>[,<variant>[,<key suffix>[,<extra bench args, + for spaces>]]]]
#                            rocprofv3 kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in their own
#                            passes (scripts/gpu_profile.sh), parsed by scripts/parse_prof.py
#   sq=<cfg>,<counters>      one rocprofv3 --pmc pass with the given SQ_ counters (<= 8), sq_<cfg>.csv
#   sqv=<cfg>,<v>,<counters> the same on plan variant <v> (bench.py --variant), sq_<cfg>_v<v>
#   kbench=<args>            fft-wavespec_amd/bin/kbench <args> (spaces as commas)
#   kalman=<args>            fft-wavespec_amd/bin/kalman_bench <args>
#   bin=<name>,<args>        fft-wavespec_amd/bin/<name> <args> (a diagnostic tool, spaces as commas)
#   harness=<args>           python scripts/<args> (a host-path timing script), spaces as commas
#   shards[=<args>]          python scripts/emulate_shards.py <tag dir>/shards.json <args> (strong-scaling shards
#                            emulated one rank at a time on this GPU), args comma-separated
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
run() {  # run <seconds> <stdout file> <stderr file> <cmd...>
    local t=$1 out=$2 err=$3
    shift 3
    if [ "$out" = "$err" ]; then
        timeout -k 10 "$t" "$@" > "$out" 2>&1
    else
        timeout -k 10 "$t" "$@" > "$out" 2> "$err"
    fi
    local rc=$?
    echo "[$TAG] rc=$rc: $*"
    if [ $rc -ne 0 ]; then
        tail -40 "$out"
        tail -20 "$err"
        exit $rc
    fi
}
for step in "$@"; do
    key=${step%%=*}
    val=""
    [ "$key" != "$step" ] && val=${step#*=}
    case $key in
    tests)
        # comma-separated pytest arguments; '+' stands for a space inside one argument (-k expressions)
        IFS=',' read -ra targs <<< "${val:-tests}"
        for i in "${!targs[@]}"; do targs[$i]=${targs[$i]//+/ }; done
        run 1100 $O/tests.log $O/tests.log python -u -m pytest "${targs[@]}" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
        tail -3 $O/tests.log
        ;;
    smoke)
        run 120 $O/smoke.log $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
        cat $O/smoke.log
        ;;
    bench|benchc)
        # benchc: the same line with the CPU baseline beside it (1 core + the job's cores, the closing check)
        cpuflag="--no-cpu-baseline"
        [ "$key" = "benchc" ] && cpuflag=""
        cfg=${val%%,*}
        extra=""
        [ "$cfg" != "$val" ] && extra=${val#*,}
        # one file per (config, arguments): repeated A/B steps do not overwrite each other
        tagx=$(echo "${extra//,/_}" | tr -c 'A-Za-z0-9_.\n-' '_')
        bf=$O/bench_$cfg${tagx:+_$tagx}
        run 300 $bf.json $bf.err python bench.py --config $cfg --steps 100 --warmup 20 $cpuflag ${extra//,/ }
        python3 -c "
import json; d=json.loads(open('$bf.json').read().strip().splitlines()[-1])
print('$cfg', '$extra', d['config'].get('algorithm'), '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
        ;;
    default)
        run 400 $O/bench_default.json $O/bench_default.err python bench.py
        cat $O/bench_default.json
        ;;
    prof)
        IFS=',' read -r cfg algo var suf extra <<< "$val"
        run 900 $O/prof_$cfg.log $O/prof_$cfg.log bash scripts/gpu_profile.sh $TAG $cfg ${algo:-auto} ${var:-0} "${suf:-}" ${extra//+/ }
        cat $O/prof_$cfg.log
        ;;
    sq)
        cfg=${val%%,*}
        ctr=${val#*,}
        run 120 $O/sq_$cfg.log $O/sq_$cfg.log rocprofv3 --pmc ${ctr//,/ } --kernel-trace --output-format csv -d $O/sq_$cfg -o run -- \
            python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline
        ;;
    sqv)
        # sqv=<cfg>,<plan variant>,<counters>: the same pass on a plan variant, sq_<cfg>_v<variant>
        cfg=${val%%,*}
        rest=${val#*,}
        var=${rest%%,*}
        ctr=${rest#*,}
        run 120 $O/sq_${cfg}_v$var.log $O/sq_${cfg}_v$var.log rocprofv3 --pmc ${ctr//,/ } --kernel-trace --output-format csv \
            -d $O/sq_${cfg}_v$var -o run -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --variant $var
        ;;
    kbench)
        run 300 $O/kbench.log $O/kbench.log fft-wavespec_amd/bin/kbench ${val//,/ }
        cat $O/kbench.log
        ;;
    kalman)
        kl=$O/kalman_bench_${val//,/_}.log
        run 300 $kl $kl fft-wavespec_amd/bin/kalman_bench ${val//,/ }
        cat $kl
        ;;
    bin)
        # any diagnostic binary of fft-wavespec_amd/bin: bin=<name>,<args>
        bn=${val%%,*}
        ba=""
        [ "$bn" != "$val" ] && ba=${val#*,}
        bl=$O/bin_${val//,/_}.log
        run 300 $bl $bl fft-wavespec_amd/bin/$bn ${ba//,/ }
        cat $bl
        ;;
    harness)
        hn=${val//,/_}
        hl=$O/harness_${hn//\//_}.log
        run 300 $hl $hl python3 scripts/${val//,/ }
        cat $hl
        ;;
    shards)
        run 1100 $O/shards.log $O/shards.log python3 -u scripts/emulate_shards.py $O/shards.json ${val//,/ }
        cat $O/shards.log
        ;;
    *)
        echo "unknown step $step"
        exit 2
        ;;
    esac
done
