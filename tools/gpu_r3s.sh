#!/bin/bash
# The round-3 check of the in-tree build (tools/gpu_r3_final.sh), then a same-box A/B of next8
# (u16 round staging positions) against it on C5 and C3.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tools/gpu_r3_final.sh r3s || exit $?
L=tools/abl/next8.so
tools/gpu_steps.sh \
  "200|r3s/ab_c5.log|bash tools/ab_mix.sh c5 1 'cur|' '$L|'" \
  "200|r3s/ab_c3.log|bash tools/ab_mix.sh c3 1 'cur|' '$L|'"
