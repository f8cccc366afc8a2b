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


# ---- --gpus N: the bench starts its own ranks; n_gpus is the GPUs asked for ----
def test_resolve_world():
    import pytest

    b = _bench()
    assert b.resolve_world(None, {}) == ("run", 1)
    assert b.resolve_world(1, {}) == ("run", 1)
    assert b.resolve_world(8, {}) == ("launch", 8)
    assert b.resolve_world(None, {"WORLD_SIZE": "4"}) == ("run", 4)   # a rehearsal launched without --gpus
    assert b.resolve_world(4, {"WORLD_SIZE": "4"}) == ("run", 4)      # the driver's torchrun form
    with pytest.raises(ValueError, match="WORLD_SIZE"):
        b.resolve_world(2, {"WORLD_SIZE": "4"})
    with pytest.raises(ValueError, match="WORLD_SIZE"):
        b.resolve_world(1, {"WORLD_SIZE": "8"})
    with pytest.raises(ValueError):
        b.resolve_world(0, {})


def test_launcher_cmd():
    import sys

    b = _bench()
    cmd = b.launcher_cmd(2, ["--gpus", "2", "--steps", "3"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(str(ROOT / "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "2", "--steps", "3"]


def _run_bench(args, env_extra, timeout=180):
    import os
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_gpus_2_launches_two_ranks():
    """`python bench.py --gpus 2` with no launcher around it starts two ranks through
    torch.distributed.run as a child (no GPU touched by the parent); each rank sees WORLD_SIZE=2.
    (--launch-probe stops every rank before its first GPU call; MTB_BENCH_ONE_DEVICE skips the device
    count, this container having no GPU.)"""
    p = _run_bench(["--gpus", "2", "--launch-probe"], {"MTB_BENCH_ONE_DEVICE": "1"})
    assert p.returncode == 0, p.stderr[-2000:]
    got = sorted(json.loads(x)["rank"] for x in p.stdout.splitlines() if x.startswith("{"))
    worlds = {json.loads(x)["world"] for x in p.stdout.splitlines() if x.startswith("{")}
    assert got == [0, 1] and worlds == {2}
    assert "torch.distributed.run" in p.stderr


def test_gpus_mismatch_raises():
    p = _run_bench(["--gpus", "2", "--launch-probe"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=4" in p.stderr
    p = _run_bench(["--gpus", "2", "--launch-probe"], {})  # no GPU here: the launcher refuses, nothing starts
    assert p.returncode != 0 and "GPU(s) visible" in p.stderr


def test_cpu_baseline_names_cpu_model(tmp_path):
    """Every cpu_baseline the bench builds carries the host's CPU model and nproc (SURVEY §8(d);
    VERDICT r05 item 7), and the stdout line keeps it."""
    import re

    b = _bench()
    src = (ROOT / "bench.py").read_text()
    built = re.findall(r'\{"value": round\([^\n]*"kind": "port"', src)
    assert len(built) >= 3 and all('"cpu_model": cpu_model()' in x for x in built)
    m = b.cpu_model()
    assert "nproc" in m
    full = json.loads((ROOT / "profiles" / "r04" / "bench_detail.json").read_text())
    full["cpu_baseline"]["cpu_model"] = m
    full["long_reads"]["cpu_baseline"]["cpu_model"] = m
    line = b.compact_line(full, str(tmp_path / "d.json"))
    assert line["cpu_baseline"]["cpu_model"] == m and line["long_reads"]["cpu_baseline"]["cpu_model"] == m


def test_random_roofline_fracs_at_most_one():
    """random_roofline prices the random kernels by the HBM bytes they move (PMC: fetched 128-B lines,
    32-B write requests) against the calibrated random 128-B-line bandwidth (the
    old request-count model put K4 at 1.02). Over every workload's committed PMC pass and kernel
    trace no frac exceeds 1; the headline's K4 sits near 0.7, K1F near its ceiling."""
    b = _bench()
    seen = 0
    for p in sorted((ROOT / "profiles" / "r05").glob("stage_traffic_*.json")):
        tf = json.loads(p.read_text())
        ms = tf["stage_ms"]["stage_ms"]
        kern = [ms.get(k, 0.0) for k in b.KERNELS_SORT]
        rr = b.random_roofline(kern, b.KERNELS_SORT, (tf, str(p)), Q=1)
        assert rr, p.name
        for k, v in rr.items():
            assert 0 < v["frac"] <= 1.0, (p.name, k, v)
            assert abs(v["frac"] - v["traffic_tb_per_s"] / v["ceiling_tb_per_s_at_128B"]) < 2e-3
            seen += 1
        if p.name == "stage_traffic_gtdb.json":
            assert 0.6 < rr["match_join"]["frac"] < 0.8 and rr["filter"]["frac"] > 0.85
    assert seen >= 10
    assert b.random_roofline([1.0] * 7, b.KERNELS_SORT, (None, None)) is None  # no PMC pass: no entry
