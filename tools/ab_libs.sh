#!/bin/bash
# A/B of library builds on bench lines, alternating (ROUNDS, default 2):
#   LIBS="name=path name2=path2 ..." CONFIGS="<bench args>;<bench args>;..." bash tools/ab_libs.sh
# (path "-" = the in-tree libsacx.so).  One line per run: round, arm, bench args, value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IFS=';' read -r -a cfgs <<< "${CONFIGS}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${cfgs[@]}"; do
    for arm in $LIBS; do
      name=${arm%%=*}; path=${arm#*=}
      if [ "$path" = "-" ]; then unset SACX_LIBPATH; else export SACX_LIBPATH=$PWD/$path; fi
      v=$(timeout -k 10 300 python bench.py $c --no-cpu-baseline --no-roofline --packed-leg 0 2>&1 | grep -o '"value": [0-9.]*')
      rc=$?; echo "$r $name [$c] $v"; [ $rc -eq 0 ] || exit 1
    done
  done
done
