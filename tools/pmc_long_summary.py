"""Per-stage HBM bytes per long-read batch from tools/pmc_long2.sh's FETCH_SIZE / WRITE_SIZE
passes: the dispatches from the first long-read batch on (the 5th k_extract_filter: the bench runs
2 short batches x (warm-up + timed) first), split into batches at k_extract_filter and into stages
as tools/stage_profile.py does; FETCH_SIZE doubled (MI355X_MICROARCH.md), WRITE_SIZE as is.
Usage: python tools/pmc_long_summary.py <fetch csv> <write csv> > profiles/r02/stage_traffic_long.json"""
import collections
import csv
import json
import sys

sys.path.insert(0, "tools")
from stage_profile import STAGES, short  # noqa: E402


def stage(k):
    if k.startswith("k_extract_filter"):
        return "filter"
    if k.startswith("k_radix") or k.startswith("k_scan") and False:
        return "kmer_sort"
    if k.startswith(("k_match<", "k_join_uniform<", "k_join_pair<")) or k == "k_join_uniform":
        return "match_join"
    if k.startswith(("k_compact_segments", "k_spill_scatter")):
        return "match_transpose"
    if k.startswith(("k_segsort", "k_thin_big", "k_pack_live", "k_max_seg", "k_merge", "k_chunk_sort")):
        return "match_sort"
    return None


def load(path, counter, scale):
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        rows.append((int(r["Dispatch_Id"]), short(r["Kernel_Name"]), float(r["Counter_Value"]) * 1024 * scale))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[1].startswith("k_extract_filter")]
    if len(starts) < 8:
        raise SystemExit(f"expected 8 batches, found {len(starts)}")
    batches = [rows[starts[b]:(starts[b + 1] if b + 1 < len(starts) else len(rows))] for b in range(4, 8)]
    tot = collections.OrderedDict((s, 0.0) for s in STAGES)
    for b in batches:
        cur = "filter"
        for _, k, v in b:
            st = stage(k)
            if st is None:  # scans / radix passes: the sort before the join, K6 after K5
                st = "kmer_sort" if cur in ("filter", "kmer_sort") else ("assign" if cur in ("match_sort", "assign") else cur)
            if k.startswith(("k_run_", "k_group_keys", "k_match_paths", "k_combine", "k_choose", "k_compact_taxcnt",
                             "k_taxcnt")):
                st = "assign"
            cur = st
            tot[st] += v / len(batches)
    return tot


f = load(sys.argv[1], "FETCH_SIZE", 2.0)
w = load(sys.argv[2], "WRITE_SIZE", 1.0)
print(json.dumps({"workload": "config-3 long reads: 25k ONT-like reads per batch (N50 ~10 kb), GTDB-scale DB "
                              "(small build), per batch (avg of 4)",
                  "source": "tools/pmc_long2.sh + tools/pmc_long_summary.py; FETCH_SIZE doubled",
                  "stages": {s: {"fetch_bytes": int(f[s]), "write_bytes": int(w[s]), "hbm_bytes": int(f[s] + w[s])}
                             for s in STAGES}}, indent=1))
