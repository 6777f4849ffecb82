#!/bin/bash
# A/B of one environment knob on the default bench (run via gpurun from the repo root):
#   gpurun -- bash scripts/ab_env.sh <tag> <VAR> "<value> <value> ..." [bench.py arguments]
# One bench line per value (headline mode only: no companion step, no CPU baseline), each under
# its own time limit, stopping at the first failure.  An empty-string value ("") leaves VAR unset.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:?tag}
VAR=${2:?variable}
VALUES=${3:?values}
shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in $VALUES; do
  echo "== $VAR=$v $(date +%T)"
  if [ "$v" = "unset" ]; then
    timeout -k 10 300 python -u bench.py --no-companion --no-cpu-baseline --steps 3 --warmup 1 "$@" \
      > "$OUT/ab_${VAR}_unset.json" 2> "$OUT/ab_${VAR}_unset.log"
  else
    env "$VAR=$v" timeout -k 10 300 python -u bench.py --no-companion --no-cpu-baseline --steps 3 \
      --warmup 1 "$@" > "$OUT/ab_${VAR}_$v.json" 2> "$OUT/ab_${VAR}_$v.log"
  fi
  rc=$?
  echo "== $VAR=$v rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
