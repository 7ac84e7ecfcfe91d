set -o pipefail
O=gpurun_out/r6ch; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_graph.py -k chain -x -q --timeout 200 --timeout-method thread > $O/chain.log 2>&1 || { echo chain failed; tail -40 $O/chain.log; exit 1; }
tail -1 $O/chain.log
timeout -k 10 900 python -u -m pytest tests -m gpu -k "train or ddp or graph_trainer" -x -q --timeout 300 --timeout-method thread > $O/train.log 2>&1 || { echo train tests failed; tail -40 $O/train.log; exit 1; }
tail -1 $O/train.log
timeout -k 10 400 python tools/train_ab.py --steps 6 --reps 6 base train.CHAIN_FUSED=0 > $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
tail -1 $O/ab.txt
timeout -k 10 300 python bench.py --model train --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_train.json 2> $O/bench_train.err || { tail $O/bench_train.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_train.json')); print('train line', d['value'], d['ms_per_step'])"
