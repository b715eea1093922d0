#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/ab_mix.sh c5 2 "cur|LMR_UNPART_SPLIT=4" "cur|LMR_UNPART_SPLIT=8" "cur|LMR_UNPART_SPLIT=16" "cur|LMR_UNPART_SPLIT=8 LMR_UNPART_NT=512"
