#!/bin/bash
# Bench A/B/A/B on one box (default tree vs the env assignment $1), for effects near the
# box's run-to-run noise.  Outputs: gpurun_out/${2:-abab}/.
set -o pipefail
O=gpurun_out/${2:-abab}; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/a$i.json 2> $O/a$i.err || { echo bench failed; tail $O/a$i.err; exit 1; }
  env $1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b$i.json 2> $O/b$i.err || { echo bench failed; tail $O/b$i.err; exit 1; }
done
python - "$O" <<'P'
import json, os, sys
for f in ("a1", "b1", "a2", "b2"):
    d = json.load(open(os.path.join(sys.argv[1], f + ".json")))
    print(f, d["value"], {k: v["avg_launch_us"] for k, v in d["roofline"]["per_entry"].items()})
P
