#!/bin/bash
# PMC passes for the merge and front kernels (each pass its own run).
set -e
export TMPDIR=/tmp
R=$PWD
KERNEL=merge_eval_kernel bash profiles/pmc_front.sh gpurun_out/pmc_eval
KERNEL=merge_write_kernel bash profiles/pmc_front.sh gpurun_out/pmc_write
KERNEL=front_kernel bash profiles/pmc_front.sh gpurun_out/pmc_front
