"""Print bench_variants.py JSON results (skipping log lines) compactly."""
import json
import sys

for path in sys.argv[1:]:
    txt = open(path).read()
    body = txt[txt.index("{"):] if "{" in txt else "{}"
    lines = [l for l in txt.splitlines() if l.startswith("PARITY")]
    d = json.loads(body)
    print(path.split("/")[-1], *lines)
    for k, v in d.items():
        print(f"  {k:12s} " + " ".join(f"{a}={b}" for a, b in v.items()))
