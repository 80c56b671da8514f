set -o pipefail
mkdir -p gpurun_out/r11
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r11/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r11/bench_default.log 2>&1 || exit 2
timeout -k 10 900 bash profiles/collect.sh r11 fp32 > gpurun_out/r11/collect.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/upd -o upd -- python3 tools/probes/gpu_update_probe.py 5 > gpurun_out/r11/update_probe.log 2>&1 || exit 4
cp /tmp/upd/upd_kernel_stats.csv gpurun_out/r11/ 2>/dev/null || find /tmp/upd -name "*kernel_stats*" -exec cp {} gpurun_out/r11/ \;
