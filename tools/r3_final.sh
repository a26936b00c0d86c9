#!/bin/bash
# Round-3 final evidence: bench.py kernel stats (8192^2 and the 1024 x 8192
# per-rank plate), smoke, the 2- and 4-rank RCCL rehearsals of the bench path.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r3final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for cfg in "8192 8192" "1024 8192"; do set -- $cfg
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/prof_$1 -o run -- python3 $OLDPWD/bench.py --nx $1 --ny $2 --steps 5 --warmup 2 > $OLDPWD/$O/prof_$1.log 2>&1 || { tail -30 $OLDPWD/$O/prof_$1.log; exit 1; }
  cd $OLDPWD; tail -1 $O/prof_$1.log | cut -c1-200
done
bash tools/rccl_rehearsal.sh "2 4" --steps 3 --warmup 1 > $O/rehearsal.log 2>&1 || { tail -30 $O/rehearsal.log; exit 1; }
cp gpurun_out/rccl_rehearsal_n2.json gpurun_out/rccl_rehearsal_n4.json $O/
grep -o '"verified": [a-z]*' $O/rccl_rehearsal_n*.json
echo done
