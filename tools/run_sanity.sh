set -o pipefail
bash tools/gpu_check.sh && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload C5 --bytes-per-gpu 4294967296 > gpurun_out/c5.log 2>&1 && tail -1 gpurun_out/c5.log | cut -c1-900 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload C4 --bytes-per-gpu 2147483648 > gpurun_out/c4.log 2>&1 ; tail -1 gpurun_out/c4.log | cut -c1-1200
