"""Print a bench line's headline and per-pass kernel times (A/B sessions)."""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(path, "unreadable:", e)
        continue
    ps = d["roofline"].get("passes", {})
    cfg = d["config"]
    print("%-34s %.3e swipes/s  %.3f ms/step  n=%d keys=%d  %s  check=%s" % (
        path.split("/")[-1], d["value"], d["ms_per_step"], cfg["swipes_per_step"], cfg["hll_keys_this_gpu"],
        " ".join("%s=%.3f" % (k, v["ms"]) for k, v in ps.items()), d.get("check", {}).get("ok")))
