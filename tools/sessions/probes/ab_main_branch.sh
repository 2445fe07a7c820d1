# A/B of the timed graph's shape in the driver's form (20 steps, 2 branches):
# two side streams (fork + join of both) against the capture stream as one
# branch and one side stream. Headline only, alternated 4 times, fresh
# processes. Prints one line per run: form value replay_median.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ab_main_branch
mkdir -p $O
for r in 1 2 3 4; do
  for mb in 0 1; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras \
      --no-cpu-baseline --main-branch $mb > $O/run_${r}_${mb}.json 2> $O/run_${r}_${mb}.err || exit 1
    python -c "import json,sys; d=json.loads(open('$O/run_${r}_${mb}.json').read().splitlines()[-1]); print($mb, d['value'], d['value_replays']['median'], d['parity'])"
  done
done
