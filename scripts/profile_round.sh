#!/usr/bin/env bash
# Round evidence: scripts/profile_case.sh for the headline and the BASELINE
# configs on their default SOR path (red-black) and, where it changed, the
# reference order. Stops at the first failure. CASES narrows the list.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=scripts/profile_case.sh
want() { [ -z "$CASES" ] || [[ " $CASES " == *" $1 "* ]]; }
{ ! want cav4k || CASE=cavity NX=4096 NY=4096 ORDER=rb KSUB="poisson_multi_kernel<0, 4, true>" SPL=4 PMC_ITERS=400 bash $P; } &&
{ ! want cav1k || CASE=cavity NX=1024 NY=1024 ORDER=rb KSUB="poisson_resident_kernel<0, 8, false>" SPL=10000 NO_PMC=1 bash $P; } &&
{ ! want ch || CASE=channel NX=4096 NY=512 ORDER=rb KSUB="poisson_resident_kernel<1, 14, false>" SPL=10000 NO_PMC=1 bash $P; } &&
{ ! want st || CASE=backwards_step NX=8192 NY=512 RE=400 ORDER=rb KSUB="poisson_open_proof_kernel<2, 4>" SPL=4 PMC_ITERS=400 bash $P; } &&
{ ! want chlex || CASE=channel NX=4096 NY=512 ORDER=lex KSUB="poisson_resident_kernel<1, 14, true>" SPL=10000 NO_PMC=1 bash $P; } &&
{ ! want cav1klex || CASE=cavity NX=1024 NY=1024 ORDER=lex KSUB="poisson_resident_kernel<0, 8, true>" SPL=10000 NO_PMC=1 bash $P; } &&
{ ! want stlex || CASE=backwards_step NX=8192 NY=512 RE=400 ORDER=lex KSUB="poisson_lexw_kernel<2, 4, false, true>" SPL=4 PMC_ITERS=5000 bash $P; } &&
{ ! want cav4klex || CASE=cavity NX=4096 NY=4096 ORDER=lex KSUB="poisson_lexw_kernel<0, 4, false, true>" SPL=4 PMC_ITERS=5000 bash $P; }
