#!/bin/bash
# rocprofv3 evidence for bench.py: kernel trace + stats, then two PMC passes
# (FETCH_SIZE, WRITE_SIZE -- separate passes, no runtime/sys trace), then a
# summary (per-kernel stats + per-launch HBM traffic of the gridding kernel).
# One stream (--no-pipeline): every gridding launch on the whole GPU, as in
# the serial pass whose HIP-event time bench.py reports as kernel_ms.
cd "$(dirname "$0")/.." || exit 1
tag=${1:-r01}
out=gpurun_out/prof_${tag}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
    python3 bench.py --steps 5 --warmup 2 --cpu-chans 0 --no-api --no-extra --no-pipeline > $out/bench_trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_grid" --output-format csv \
    -d $out/fetch -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-chans 0 --no-api --no-extra --no-pipeline > $out/bench_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_grid" --output-format csv \
    -d $out/write -o run -- python3 bench.py --steps 1 --warmup 1 --cpu-chans 0 --no-api --no-extra --no-pipeline > $out/bench_write.log 2>&1 || exit $?
python3 scripts/summarize_profile.py $out > $out/summary.txt && cat $out/summary.txt
