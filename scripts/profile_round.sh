#!/usr/bin/env bash
# Round evidence: scripts/profile_case.sh for the headline and the open-case
# BASELINE configs (red-black and the reference's order). Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=scripts/profile_case.sh
CASE=cavity NX=4096 NY=4096 ORDER=rb KSUB="poisson_multi_kernel<0, 4, true>" SPL=4 PMC_ITERS=400 bash $P &&
CASE=cavity NX=4096 NY=4096 ORDER=lex KSUB="poisson_lexw_kernel<0, 4, false, true>" SPL=4 PMC_ITERS=5000 bash $P &&
CASE=channel NX=4096 NY=512 ORDER=rb KSUB="poisson_multi_kernel<1, 2, false>" SPL=2 PMC_ITERS=400 bash $P &&
CASE=channel NX=4096 NY=512 ORDER=lex KSUB="poisson_lexw_kernel<1, 4, false, true>" SPL=4 PMC_ITERS=3000 bash $P &&
CASE=backwards_step NX=8192 NY=512 RE=400 ORDER=rb KSUB="poisson_multi_kernel<2, 2, false>" SPL=2 PMC_ITERS=400 bash $P
[ $? -eq 0 ] && CASE=backwards_step NX=8192 NY=512 RE=400 ORDER=lex KSUB="poisson_lexw_kernel<2, 4, false, true>" SPL=4 PMC_ITERS=5000 bash $P
