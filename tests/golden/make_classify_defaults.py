"""Regenerate tests/golden/classify_defaults.json from the reference's own text.

Runs in this container only (it reads /root/reference, which the GPU box does not have); the
committed JSON is what tests/test_abi.py reads. The numeric and boolean assignments of
setClassifyDefaults (/root/reference/src/workflow/classify.cpp:10-37) are parsed as written, each
with its line number; commented-out lines are skipped.
"""
import json
import pathlib
import re

HERE = pathlib.Path(__file__).resolve().parent
REF = pathlib.Path("/root/reference/src/workflow/classify.cpp")


def parse(text: str):
    lines = text.split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"\s*void\s+setClassifyDefaults\s*\(", l))
    out = {}
    for i in range(start + 1, len(lines)):
        l = lines[i].split("//")[0]
        if lines[i].strip().startswith("}"):
            break
        m = re.match(r"\s*par\.(\w+)\s*=\s*([^;]+);", l)
        if not m:
            continue
        v = m.group(2).strip()
        if v in ("true", "false"):
            val = v == "true"
        elif re.fullmatch(r"-?\d+", v):
            val = int(v)
        elif re.fullmatch(r"-?\d*\.\d+", v):
            val = float(v)
        else:
            continue  # strings (taxonomyPath)
        out[m.group(1)] = {"value": val, "line": i + 1}
    return out


def main():
    d = parse(REF.read_text())
    assert "minConsCnt" in d and "tieRatio" in d, d
    (HERE / "classify_defaults.json").write_text(json.dumps(
        {"source": "setClassifyDefaults, src/workflow/classify.cpp (parsed by make_classify_defaults.py)",
         "defaults": d}, indent=1) + "\n")
    print(f"{len(d)} defaults")


if __name__ == "__main__":
    main()
