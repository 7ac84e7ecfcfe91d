set -o pipefail
O=gpurun_out/trab; mkdir -p $O
[ -n "$SKIP_TESTS" ] || { timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "train" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }; }
[ -n "$SKIP_TESTS" ] || tail -1 $O/t.log
for v in "HREG_TRAIN_B6=0" "HREG_TRAIN_B6=1" "HREG_TRAIN_B6_MIN_N=0" "HREG_TRAIN_B6=0" "HREG_TRAIN_B6=1" "HREG_TRAIN_B6_MIN_N=0"; do
  env $v timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b.json')); print('$v', d['value'], d['ms_per_step'])"
done
