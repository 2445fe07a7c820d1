#!/bin/bash
# r06au: the final tree (no spill in any frame geometry)
# (after r06ai): the whole GPU suite (verbose), smoke, and the
# default bench for the frame and segmentation figures.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r06au
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1
rc=$?
tail -2 $OUT/pytest.log; tail -1 $OUT/smoke.log
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06au/bench.json"))
ex = d["extras"]
print(json.dumps({"value": d["value"], "frac": d["roofline"]["frac"],
                  "validate": ex["frames_validate_F1514"]["frac_of_peak"],
                  "validate_4br": ex["frames_validate_F1514"]["pipeline"]["frac_of_peak"],
                  "fields": ex["frames_generate_fields_F1514"]["frac_of_peak"],
                  "generate": ex["frames_generate_F1514"]["frac_of_peak"],
                  "zc_1024": ex["burst_latency_host"]["bursts"]["1024"]["zero_copy"]["us_median"],
                  "segment": ex["segment_TSO_64K_mss1460"]["frac_of_peak"],
                  "segment_4br": ex["segment_TSO_64K_mss1460"]["pipeline"]["frac_of_peak"],
                  "segment_counted": ex["segment_TSO_64K_mss1460"]["device_counted"]["frac_of_peak"]}))
PY
exit $rc
