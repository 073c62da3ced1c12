#!/bin/bash
# GPU box: bench.py at 8 and 16 waveforms per launch, 3 rotated rounds (r05zb).
#   bash tools/gpu/ab_batch.sh
set -o pipefail
O=gpurun_out/r05zb; mkdir -p $O
for r in 1 2 3; do
  for b in 8 16; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --warmup 5 --batch $b > $O/b${b}_$r.json 2> $O/b${b}_$r.err || { tail -5 $O/b${b}_$r.err; exit 2; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('AB', sys.argv[2], sys.argv[3], round(d['value'],1), round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms'],3))" $O/b${b}_$r.json $b $r
  done
done
