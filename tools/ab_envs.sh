#!/bin/bash
# A/B of environment settings on bench lines, alternating (ROUNDS, default 2):
#   ENVS="name=VAR=val,VAR2=val2 name2=VAR=val ..." CONFIGS="<bench args>;..." bash tools/ab_envs.sh
# (an arm "name=" sets nothing).  One line per run: round, arm, bench args, value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS=';' read -r -a cfgs <<< "${CONFIGS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${cfgs[@]}"; do
    for arm in $ENVS; do
      name=${arm%%=*}; sets=${arm#*=}
      v=$(env ${sets//,/ } timeout -k 10 300 python bench.py $c --no-cpu-baseline --no-roofline --packed-leg 0 2>&1 | grep -o '"value": [0-9.]*')
      rc=$?; echo "$r $name [$c] $v"; [ $rc -eq 0 ] || exit 1
    done
  done
done
