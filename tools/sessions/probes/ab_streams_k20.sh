# A/B of the timed graph's branch count in the driver's form (20 steps) with
# the 32 x 3 F1500 kernel: 1, 2, 3 and 4 branches alternated 4 times in
# fresh processes, headline only. Prints: streams value replay_median.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_streams_k20
mkdir -p $O
for r in 1 2 3 4; do
  for k in 1 2 3 4; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras \
      --no-cpu-baseline --streams $k > $O/run_${r}_${k}.json 2> $O/run_${r}_${k}.err || exit 1
    python -c "import json; d=json.loads(open('$O/run_${r}_${k}.json').read().splitlines()[-1]); print($k, d['value'], d['value_replays']['median'], d['parity'])"
  done
done
