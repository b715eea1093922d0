#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 600 bash tools/ab_mix.sh c2 2 "cur|" "cur|LMR_FT_GROUP=1" "cur|LMR_FT_GROUP=2" "cur|LMR_FT_GROUP=4" "cur|LMR_FT_GROUP=8"
