"""Summarise bench.py JSON lines of A/B logs: value, CNN ms, post ms per file (sorted by name)."""
import glob
import json
import sys

for pat in sys.argv[1:]:
    for f in sorted(glob.glob(pat)):
        try:
            line = [x for x in open(f) if x.startswith("{")][-1]
        except (IndexError, OSError):
            print("%-48s (no result)" % f)
            continue
        d = json.loads(line)
        r = d.get("roofline") or {}
        pr = d.get("post_roofline") or r
        print("%-48s %10.2f fps  cnn %7.3f ms  post %6.3f ms" % (
            f, d["value"], r.get("avg_launch_ms", float("nan")) if d.get("post_roofline") else float("nan"),
            pr.get("avg_launch_ms", float("nan"))))
