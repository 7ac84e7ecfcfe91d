"""print value / ms_per_step / roofline.frac of bench JSON lines: ab_lines_print.py DIR NAME..."""
import json
import sys

d = sys.argv[1]
for name in sys.argv[2:]:
    j = json.load(open(f"{d}/{name}.json"))
    print(name, j["value"], j["ms_per_step"], (j.get("roofline") or {}).get("frac"))
