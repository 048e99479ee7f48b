#!/bin/bash
# PMC counters of the final build's main kernels on the M2 bench.
cd $GRAFT_REPO_ROOT
bash tools/pmc_kernels.sh pmc_final_bwd bwd2_kernel || exit 1
bash tools/pmc_kernels.sh pmc_final_shadam sh_bwd_staged || exit 2
