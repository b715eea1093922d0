#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 600 bash tools/ab_mix.sh c2 2 "cur|" "cur|LMR_FREE=0 LMR_STAGED=1 LMR_STAGE_SPLIT=32" "cur|LMR_FREE=0 LMR_STAGED=1 LMR_STAGE_SPLIT=16" "cur|LMR_FREE=0 LMR_STAGED=0" &&
timeout -k 10 600 bash tools/ab_mix.sh c3 2 "cur|" "cur|LMR_STAGED=1 LMR_STAGE_SPLIT=8" "cur|LMR_STAGED=1 LMR_STAGE_SPLIT=4"
