#!/bin/bash
# round-2 PMC passes: front kernel, merge_eval, ans_encode (each pass its own run)
set -e
export TMPDIR=/tmp
KERNEL=front_kernel bash profiles/pmc_front.sh gpurun_out/pmc2_front
KERNEL=merge_eval_kernel bash profiles/pmc_front.sh gpurun_out/pmc2_eval
KERNEL=ans_encode_kernel bash profiles/pmc_front.sh gpurun_out/pmc2_ans
