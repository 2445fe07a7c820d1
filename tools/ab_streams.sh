set -e
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for r in 0 1 2 3; do for s in 4 8 4 8; do
  timeout -k 10 120 python bench.py --no-extras --no-cpu-baseline --streams $s > gpurun_out/s3.json 2>/dev/null
  python -c "import json;d=json.loads(open('gpurun_out/s3.json').read().splitlines()[-1]);print($r,$s,d['value'],d['value_replays']['median'],d['roofline']['avg_launch_us'],flush=True)" | tee -a gpurun_out/streams3.log
done; done
