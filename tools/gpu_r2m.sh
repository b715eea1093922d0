#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/ab_mix.sh c3 2 "tools/abl/base.so|" "cur|" "cur|LMR_UNPART_SPLIT=4" "cur|LMR_UNPART_NT=256 LMR_UNPART_SPLIT=4" "cur|LMR_UNPART_U=8" "cur|LMR_UNPART_U=2 LMR_UNPART_SPLIT=2" &&
timeout -k 10 900 bash tools/ab_mix.sh c5 2 "cur|" "cur|LMR_UNPART_SPLIT=4" "cur|LMR_UNPART_NT=256 LMR_UNPART_SPLIT=4" "cur|LMR_UNPART_U=8"
