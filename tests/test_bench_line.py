"""bench.py's stdout line stays parseable by the driver (a 20.8-KB line overflowed
its ~15.5-KB stdout capture): under LINE_CAP with the headline fields, roofline and cpu_baseline, the
full tree in the detail file it names."""
import importlib.util
import json
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_compact_line_under_cap(tmp_path):
    b = _bench()
    full = json.loads((ROOT / "profiles" / "r03" / "bench_default.json").read_text())
    detail = tmp_path / "detail.json"
    line = b.compact_line(full, str(detail))
    s = json.dumps(line)
    assert len(s) <= b.LINE_CAP
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline", "parity_sample", "long_reads"):
        assert k in line, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"], k
    assert line["long_reads"]["parity_sample"] is True
    assert json.loads(detail.read_text()) == full


def test_compact_line_drops_summaries_before_headline(tmp_path):
    b = _bench()
    full = json.loads((ROOT / "profiles" / "r03" / "bench_default.json").read_text())
    # an oversized summary section is dropped, the headline fields stay
    full["variants"] = {f"v{i}": dict(full["variants"]["related"], value=i) for i in range(200)}
    line = b.compact_line(full, str(tmp_path / "d.json"))
    assert len(json.dumps(line)) <= b.LINE_CAP
    assert "variants" not in line
    assert line["roofline"]["frac"] == full["roofline"]["frac"]
    assert line["cpu_baseline"]["value"] == full["cpu_baseline"]["value"]


def test_round4_detail_round_trips(tmp_path):
    """This round's full detail (profiles/r04/bench_detail.json) compacts to the committed line's
    fields, the CPU baseline's sample text whole."""
    b = _bench()
    full = json.loads((ROOT / "profiles" / "r04" / "bench_detail.json").read_text())
    line = b.compact_line(full, str(tmp_path / "d.json"))
    assert len(json.dumps(line)) <= b.LINE_CAP
    assert line["cpu_baseline"]["sample"] == full["cpu_baseline"]["sample"]
    assert line["end_to_end"]["bgzf"]["tsv_matches_oracle"] is True
    assert line["cold_run"]["tsv_matches_oracle"] is True


def test_variant_batches():
    """Per-variant QuerySplits unless --variant-batch names one for all."""
    b = _bench()

    class A:
        variant_batch = 0

    assert b.variant_batch(A, "related") == 2_000_000
    assert b.variant_batch(A, "syncmer") == b.variant_batch(A, "conserved") == 3_333_334
    A.variant_batch = 1_000_000
    assert b.variant_batch(A, "syncmer") == 1_000_000


def test_workload_labels_follow_parameters():
    """config.workload is built from the run's own numbers: a 1M-pair, 2G-k-mer
    rehearsal can no longer call itself "config 3: 10M ... ~12G k-mers", nor a 48-GB DB larger than
    one GPU's HBM."""
    import re

    b = _bench()
    assert [b.count_label(x) for x in (10_000_000, 3_333_334, 200_000, 12.0e9, 1_000_000, 125_000)] == \
        ["10M", "3.33M", "200k", "12.0G", "1M", "125k"]
    for pairs, kmers in ((10_000_000, 12.02e9), (1_000_000, 2.0e9), (250_000, 9.8e8)):
        lab = b.config3_label(pairs, 150, int(kmers), 129_671, 500_000)
        m = re.match(r"config 3: (\S+) x 150bp .*\((\S+) k-mers, 129,671-species", lab)
        assert m and m.group(1) == b.count_label(pairs) and m.group(2) == b.count_label(int(kmers)), lab
    assert "more than one GPU" in b.config5_label(10_000_000, 150, int(35e9), 8)
    small = b.config5_label(1_000_000, 150, int(4e9), 4)  # 48 GB of records
    assert "fits one GPU" in small and "1M x 150bp" in small and "4.0G-k-mer" in small
