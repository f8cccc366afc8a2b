"""Regenerate tests/golden/genetic_code.json from the reference's own GeneticCode.h.

Runs oracle/_ref/refdump (built by `make -C oracle ref`, which compiles
/root/reference/src/commons/GeneticCode.h in place) and stores its JSON output. Only works in the
container where /root/reference is mounted; the committed JSON is what the tests read.
"""
import json
import pathlib
import subprocess

HERE = pathlib.Path(__file__).resolve().parent
ROOT = HERE.parents[1]

if __name__ == "__main__":
    subprocess.run(["make", "-C", str(ROOT / "oracle"), "ref"], check=True)
    out = subprocess.run([str(ROOT / "oracle" / "_ref" / "refdump")], check=True, capture_output=True, text=True).stdout
    data = json.loads(out)
    (HERE / "genetic_code.json").write_text(json.dumps(data, separators=(",", ":")) + "\n")
    print("wrote", HERE / "genetic_code.json")
