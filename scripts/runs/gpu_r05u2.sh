#!/bin/bash
# Round-5 GPU call U2: A0 upload by k host threads on their own streams
# (MAMG_UPLOAD_THREADS 1 / 2 / 4, alternating), bench setup phases.
OUT=$(pwd)/gpurun_out/r05u2
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -1 "$OUT/$name.log" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); st=d['setup']; print(d['value'], st['wall_s'], st['phases_ms']['upload_A0'], st['phases_ms']['setup_total'])"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
B="python -u bench.py --cpu-sample 0 --pcg 0 --compare-profiles 0 --steps 5 --no-breakdown"
for r in a b; do
  for k in 1 2 4; do MAMG_UPLOAD_THREADS=$k step u$k$r 300 $B; done
done
echo "== done"
