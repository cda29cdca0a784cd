set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for lib in default devlib/libalipmpc_dd2.so devlib/libalipmpc_dd22.so; do
  if [ $lib = default ]; then unset ALIPMPC_LIB; else export ALIPMPC_LIB=$R/$lib; fi
  for a in "16384 3 5 0" "16384 5 5 5"; do
    echo -n "$lib $a: "; timeout -k 10 120 python $R/tools/dd_bench.py $a 2>/dev/null | tail -1 || exit 1
  done
done
