"""One-line summary of a bench.py JSON line: value, per-step time, roofline, parity, secondaries."""
import json
import sys

for path in sys.argv[1:]:
    lines = [l for l in open(path) if l.startswith("{")]
    if not lines:
        print(path, "no JSON line")
        continue
    d = json.loads(lines[-1])
    r = d.get("roofline") or {}
    par = (d.get("parity") or {}).get("mismatches")
    out = {"cfg": d["config"]["workload"][:3], "n": d["n_gpus"], "value": d["value"], "ms": d["ms_per_step"],
           "kernel_ms": r.get("kernel_ms"), "bound": r.get("bound"), "frac": r.get("frac"), "mism": par}
    for k in ("batched", "e2e_host", "c2_reference_defaults"):
        if k in d:
            out[k] = d[k].get("value")
    if "post_processing" in d:
        out["post"] = {k: v for k, v in d["post_processing"].items() if k.endswith("_ms")}
    if "cpu_baseline" in d:
        cb = d["cpu_baseline"]
        out["cpu"] = (cb["value"], cb["cores"])
    print(path.split("/")[-1], json.dumps(out))
