#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/ab_mix.sh c5 2 "cur|" "cur|LMR_G_ROUND=1" && timeout -k 10 600 bash tools/ab_mix.sh c3 1 "cur|" "cur|LMR_G_ROUND=1"
