# round-5 session y: where the F1500 kernel's serial gap to its own load
# pattern goes - a diagnostic build that computes every result but stores
# none (nostore; parity is not comparable, so probe_fixed_ab runs with
# NO_PARITY), and nontemporal result stores (tools/probe_fixed.py, PROBE_NT
# 1 = nt loads, 3 = nt loads + nt stores).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05y
mkdir -p $O
ROUNDS=5 NO_PARITY=1 PROBE_LENS=1500 LIB_B=ab/abx_ck_nostore.so timeout -k 10 300 python -u tools/probe_fixed_ab.py > $O/nostore.log 2>&1 &&
ROUNDS=5 PROBE_NT=1,3 PROBE_GEOMS=32:3:256 PROBE_LENS=1500 timeout -k 10 300 python -u tools/probe_fixed.py > $O/ntstore.log 2>&1
rc=$?; grep serial_frac $O/nostore.log; tail -3 $O/ntstore.log; exit $rc
