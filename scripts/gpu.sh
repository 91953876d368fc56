#!/bin/bash
# One parameterised GPU-box runner (replaces the one-shot scripts/r03*.sh and profiles/run_s*.sh).
#
#   bash scripts/gpu.sh <tag> <step> [<step> ...]
#
# Output goes to gpurun_out/<tag>/.  Steps run in order, each under its own time limit; the first
# step that fails (test failure, abort, fault, time limit) ends the run with its exit status, so no
# further GPU work starts after trouble.  Steps:
#   tests[=<pytest -k expr>]   GPU parity tests (pytest -m gpu)            -> pytest.log
#   smoke                      __graft_entry__.smoke()                       -> smoke.log
#   bench[=<args>]             python bench.py <args> (',' separates args)   -> bench[_<n>].json / .err
#   profile[=<args>]           rocprofv3 kernel trace + stats of bench.py    -> prof_<tag>/ (profiles/run_profile.sh)
#   pmc[=<args>]               separate rocprofv3 --pmc passes of bench.py   -> prof_<tag>/ (profiles/pmc_extra.sh)
#   tiles[=<args>]             profiles/tile_scaling.py <args>               -> tiles[_<n>].json / .log
#   ab=<args>                  profiles/ab_inproc.py <args> (in-process A/B of library builds) -> ab[_<n>].txt
#   py=<script>[,<args>]       python <script> <args>                        -> py_<n>.log
#   benchgloo=<args>           BENCH_DIST_BACKEND=gloo python bench.py <args> (e.g. --gpus,2: N ranks rehearsed on one GPU)
#   trace=<args>               rocprofv3 kernel trace of profiles/render_tile.py <args> -> trace_<n>/ + trace_<n>.txt
#                              (profiles/tile_trace.py: per-kernel spans of the last render)
# Example: bash scripts/gpu.sh r04a tests smoke bench bench=--config,bunny tiles=--config,dragon
set -o pipefail
TAG=${1:?usage: scripts/gpu.sh <tag> <step>...}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for step in "$@"; do
    n=$((n + 1))
    name=${step%%=*}
    arg=""
    [[ "$step" == *=* ]] && arg=${step#*=}
    args=${arg//,/ }
    echo "[gpu.sh] step $n: $step" >&2
    case "$name" in
    tests)
        k=()
        [ -n "$arg" ] && k=(-k "$arg")
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
            > "$OUT/pytest${arg:+_$n}.log" 2>&1 ;;
    smoke)
        timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench)
        sfx=""; [ -n "$arg" ] && sfx="_$n"
        timeout -k 10 600 python -u bench.py $args > "$OUT/bench$sfx.json" 2> "$OUT/bench$sfx.err" ;;
    profile)
        bash profiles/run_profile.sh "$TAG" ${args:---steps 3 --no-cpu-baseline} ;;
    pmc)
        bash profiles/pmc_extra.sh "$TAG" ${args:---steps 3 --no-cpu-baseline} ;;
    tiles)
        sfx=""; [ -n "$arg" ] && sfx="_$n"
        timeout -k 10 600 python -u profiles/tile_scaling.py $args > "$OUT/tiles$sfx.json" 2> "$OUT/tiles$sfx.log" ;;
    ab)
        timeout -k 10 900 python -u profiles/ab_inproc.py $args > "$OUT/ab_$n.txt" 2>&1 ;;
    py)
        timeout -k 10 600 python -u $args > "$OUT/py_$n.log" 2>&1 ;;
    benchgloo)
        BENCH_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py $args > "$OUT/benchgloo_$n.json" 2> "$OUT/benchgloo_$n.err" ;;
    trace)
        timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_$n" -o run -- \
            python3 profiles/render_tile.py $args > "$OUT/trace_$n.log" 2>&1 &&
            python3 profiles/tile_trace.py "$OUT/trace_$n" > "$OUT/trace_$n.txt" ;;
    *)
        echo "[gpu.sh] unknown step '$step'" >&2
        exit 2 ;;
    esac
    rc=$?
    if [ $rc -ne 0 ]; then
        echo "[gpu.sh] step $n ($step) failed with status $rc: stopping" >&2
        exit $rc
    fi
done
