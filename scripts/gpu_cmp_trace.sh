cd /root/repo && export TMPDIR=/tmp
for w in 1 0; do
  mkdir -p gpurun_out/trw$w
  SDP_HIP_NO_WINDOW=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trw$w -o run -- python3 scripts/gpu_sweep.py SDP_HIP_DBG 0 > gpurun_out/trw$w/log.txt 2>&1 || exit 1
done
