# round-5 session x: fixed-length checksum kernel A/B (tools/probe_fixed_ab.py):
# the tree against late boundary masks (lm: the head/tail mask math kept
# behind the chunk loads instead of hoisted ahead of them), the side-input
# loads gated on the mode (sg), and both (lmsg).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05x
mkdir -p $O
ROUNDS=5 LIB_B=ab/abx_ck_lm.so,ab/abx_ck_sg.so,ab/abx_ck_lmsg.so timeout -k 10 400 python -u tools/probe_fixed_ab.py > $O/fixed_ab.log 2>&1
rc=$?; grep serial_frac $O/fixed_ab.log; exit $rc
