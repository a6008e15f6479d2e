set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g49
for k in 0 1 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/g49/b_$k.json 2> gpurun_out/g49/b_$k.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/g49/b_$k.json').read().strip().splitlines()[-1]);print('kernarg=$k', d['value'], d['roofline']['avg_launch_ms'], d['ms_per_step'], d['sorted_result']['value'])"
done
