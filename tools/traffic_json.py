"""profiles/r0N/stage_traffic_<workload>.json from one tools/measure_r0N.sh workload directory: the
per-stage HBM bytes (stage_bytes.json: FETCH_SIZE doubled per MI355X_MICROARCH.md + WRITE_SIZE) of
the profiled batch, keyed by the DB size and batch shape bench.py matches them on."""
import json
import os
import sys

w, d, batch = sys.argv[1], sys.argv[2], int(sys.argv[3])
lines = [l for l in open(os.path.join(d, "bench.json")).read().splitlines() if l.startswith("{")]
b = json.loads(lines[-1])
stages = json.load(open(os.path.join(d, "stage_bytes.json")))
stage_ms = json.load(open(os.path.join(d, "stage_time.json")))
# profiles taken before stage_profile.py named the fused k_extract_filter "filter" list it (and the
# K0 kernels, < 1 MB) as "extract": relabel, as bench.py times the fused kernel as the filter
if stages["filter"]["hbm_bytes"] == 0 and stages["extract"]["hbm_bytes"] > 0:
    stages["filter"], stages["extract"] = stages["extract"], {k: 0 for k in stages["extract"]}
    stage_ms["stage_ms"]["filter"], stage_ms["stage_ms"]["extract"] = stage_ms["stage_ms"]["extract"], 0.0
out = {"workload": w, "kmers": b["config"]["db_kmers"], "batch": batch,
       "source": f"rocprofv3 --kernel-trace (stage_time) and separate --pmc FETCH_SIZE / WRITE_SIZE passes of one "
                 f"{w} batch after a warm-up batch (tools/measure_r05.sh, tools/stage_profile.py); FETCH_SIZE doubled "
                 f"per MI355X_MICROARCH.md; the fused K1 + K1F kernel (k_extract_filter) is the filter stage",
       "stages": stages, "stage_ms": stage_ms}
print(json.dumps(out, indent=1))
