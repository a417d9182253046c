# same-box A/B of the host messages, then the quick GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
AB_STEPS=20 AB_CASES="e8:--emulate-rank 0/8|c1:--config 1|c3:--config 3" AB_VARS="msg:|nomsg:LFE_HOST_MSG=0" bash tools/ab_env.sh || exit $?
bash tools/r6_quick.sh
