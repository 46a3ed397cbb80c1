#!/bin/bash
# One build -> measure iteration on the GPU box: GPU tests, the bench line and
# a kernel trace of a short bench run, then the last batch's per-pass times.
# Usage (on the box): bash scripts/iter.sh
set -u
STEPS="tests bench prof" bash scripts/gpu_session.sh || exit $?
python scripts/last_batch.py gpurun_out/prof/run_kernel_trace.csv
