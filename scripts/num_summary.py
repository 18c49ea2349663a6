"""Summarise a MACBF_NUM_LOG file: worst measured relative error per test (and its bound)."""
import json
import sys
from collections import defaultdict

worst = defaultdict(lambda: (0.0, "", 0.0))
for line in open(sys.argv[1]):
    d = json.loads(line)
    if d["err"] >= worst[d["test"]][0]:
        worst[d["test"]] = (d["err"], d["name"], d["bound"])
for t, (e, n, b) in sorted(worst.items()):
    print(f"{e:9.2e}  bound {b:7.1e}  x{b / max(e, 1e-30):7.1f}  {t}  [{n}]")
