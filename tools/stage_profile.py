"""Per-stage GPU time and HBM traffic of one classify step, from rocprofv3 output.

Dispatches are attributed to the pipeline stages bench.py reports (kernel_ms) by their order
within a step: a step starts at k_read_meta; extract = up to and including k_extract; filter =
k_filter; kmer_sort = everything from there to the join; match_join = k_match_windows + k_match (or k_join_uniform)
(probe_join = k_probe on MTB_JOIN=probe), with the per-read count scan and a rerun if the staging
buffer grew; match_transpose = k_match_transpose or k_compact_segments (direct join); match_sort = k_segsort_* (+ the live-match scan
and k_pack_live); assign = the rest of
the step (K6 kernels, scans and taxcnt compaction).

Usage:
  python tools/stage_profile.py time  <run_kernel_trace.csv> <step index>
  python tools/stage_profile.py bytes <fetch run_counter_collection.csv> <write run_counter_collection.csv> <step index>
(bench.py default: steps 0-1 are warmup, 2-6 timed 150 bp steps; with --steps 1 --warmup 0 step 0)
FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE is doubled (MI355X_MICROARCH.md: on gfx950 it
counts half the bytes of a wide coalesced read), WRITE_SIZE is taken as is.
"""
import collections
import csv
import json
import sys

STAGES = ["extract", "filter", "kmer_sort", "match_join", "probe_join", "match_transpose", "match_sort", "assign"]


def short(name):
    return name.split("(")[0].replace("void ", "").replace("mtb::", "").strip()


def stage_of(seq):
    """seq: kernel short names of one step in dispatch order -> stage name per dispatch."""
    out = []
    stage = "extract"
    after_extract = False
    for k in seq:
        if stage == "post":
            out.append(stage)
            continue
        if k.startswith("k_read_meta"):
            stage, after_extract = "extract", False
        elif k.startswith("k_extract_filter"):  # the fused K1 + K1F: bench.py times it as the filter
            stage, after_extract = "filter", True
        elif k.startswith("k_extract"):
            stage, after_extract = "extract", True
        elif k.startswith("k_filter"):
            stage = "filter"
        elif (k.startswith(("k_match_windows", "k_prefix_firsts", "k_suffix_min", "k_tile_queries", "k_sweep"))
              or k.startswith(("k_match<", "k_join_uniform<", "k_join_pair<")) or k in ("k_match", "k_join_uniform")):  # K4 or K4S (the sweep's query starts + sweep)
            stage = "match_join"
        elif k == "k_probe" or k.startswith("k_probe<"):
            stage = "probe_join"
        elif k.startswith(("k_match_transpose", "k_compact_segments", "k_spill_scatter")):
            stage = "match_transpose"
        elif k.startswith(("k_segsort", "k_max_seg", "k_pack_live", "k_chunk_sort", "k_merge_tiles", "k_merge_finish",
                           "k_thin_big", "k_size_lists")):
            stage = "match_sort"
        elif stage == "match_sort" and not k.startswith("k_scan"):  # K5's live-count scan stays in K5
            stage = "assign"
        elif (stage == "extract" and after_extract) or stage == "filter":
            stage = "kmer_sort"
        out.append(stage)
        if k.startswith("k_compact_taxcnt"):
            stage = "post"  # the step's last kernel; later dispatches (e.g. a DB open) are not the step's
    return out


def pick_step(rows, nth):
    """rows: (dispatch_id, short_name, payload) sorted by dispatch; returns the nth step (a step
    starts at k_read_meta and runs to the next one)."""
    starts = [i for i, r in enumerate(rows) if r[1].startswith("k_read_meta")] + [len(rows)]
    return rows[starts[nth]:starts[nth + 1]]


def main():
    mode = sys.argv[1]
    if mode == "time":
        rows = []
        for r in csv.DictReader(open(sys.argv[2])):
            if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
                continue
            rows.append((int(r["Dispatch_Id"]), short(r["Kernel_Name"]),
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
        rows.sort()
        step = pick_step(rows, int(sys.argv[3]))
        st = stage_of([r[1] for r in step])
        tot = collections.OrderedDict((s, 0.0) for s in STAGES)
        kern = collections.defaultdict(float)
        for (d, k, ms), s in zip(step, st):
            if s == "post":
                continue
            tot[s] += ms
            kern[(s, k)] += ms
        print(json.dumps({"stage_ms": {k: round(v, 3) for k, v in tot.items()},
                          "kernels": {f"{s}/{k}": round(v, 3) for (s, k), v in sorted(kern.items())}}, indent=1))
    else:
        res = {}
        for path, counter, scale in ((sys.argv[2], "FETCH_SIZE", 2.0), (sys.argv[3], "WRITE_SIZE", 1.0)):
            rows = []
            for r in csv.DictReader(open(path)):
                if r["Counter_Name"] != counter:
                    continue
                rows.append((int(r["Dispatch_Id"]), short(r["Kernel_Name"]), float(r["Counter_Value"]) * 1024 * scale))
            rows.sort()
            step = pick_step(rows, int(sys.argv[4]))
            st = stage_of([r[1] for r in step])
            tot = collections.OrderedDict((s, 0.0) for s in STAGES)
            for (d, k, b), s in zip(step, st):
                if s != "post":
                    tot[s] += b
            res[counter] = tot
        out = {s: {"fetch_bytes": int(res["FETCH_SIZE"][s]), "write_bytes": int(res["WRITE_SIZE"][s]),
                   "hbm_bytes": int(res["FETCH_SIZE"][s] + res["WRITE_SIZE"][s])} for s in STAGES}
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
