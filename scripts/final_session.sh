#!/bin/bash
# Round-end evidence in one call: kernel stats + PMC passes + traffic summary +
# bench line that reads it (prof_session.sh), then GPU tests and smoke.
set -u
OUT=${OUT:-gpurun_out/final}
export OUT
bash scripts/prof_session.sh || exit $?
STEPS="tests smoke" bash scripts/gpu_session.sh
