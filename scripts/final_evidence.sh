#!/bin/bash
# The round's evidence at one build: GPU tests, the full bench, rocprofv3 --kernel-trace --stats of
# the same bench command (+ the profiling pass's own dispatches), PMC traffic / SQ split of the
# headline kernels and of the LM kernels. Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${TAG:?}
TAG=$T bash scripts/gpu_check.sh || exit $?
grep -q "stopping" gpurun_out/$T/steps.log && exit 1
TAG=${T}_pmc SQ=1 bash scripts/pmc.sh || exit $?
TAG=${T}_pmclm bash scripts/pmc_lm.sh || exit $?
