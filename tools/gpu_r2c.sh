#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/ab_mix.sh c2 2 "tools/libs/base.so|" "cur|" "cur|LMR_FINE_NT=1024 LMR_FINE_RPT=12" "cur|LMR_FINE_NT=1024 LMR_FINE_RPT=8" "cur|LMR_FINE_NT=1024 LMR_FINE_RPT=10"
