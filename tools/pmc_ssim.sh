#!/bin/bash
cd $GRAFT_REPO_ROOT
bash tools/pmc_kernels.sh pmc_ssim_f ssim || exit 1
GSPLAT_HIP_SSIM_FUSED=0 bash tools/pmc_kernels.sh pmc_ssim_u ssim || exit 2
