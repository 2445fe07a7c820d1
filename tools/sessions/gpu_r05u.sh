# round-5 session u: Toeplitz RSS A/B (tools/probe_rss.py) - the tree's kernel
# against nontemporal stores (ntst), nontemporal loads and stores (ntldst), the
# loop software-pipelined one tuple group ahead (pf, + nt stores), and 4,096
# blocks (b4k, + nt stores).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05u
mkdir -p $O
ROUNDS=3 LIB_B=ab/abx_rss_ntst.so,ab/abx_rss_ntldst.so,ab/abx_rss_pf.so,ab/abx_rss_b4k.so timeout -k 10 300 python -u tools/probe_rss.py > $O/rss_ab.log 2>&1
rc=$?; tail -2 $O/rss_ab.log; exit $rc
