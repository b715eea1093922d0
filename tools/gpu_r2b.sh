#!/bin/bash
# round-2 check: full -m gpu suite (all failures listed), then C5 / C3 benches with verification
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2b; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/gputest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 > $O/c5.log 2>&1; rc=$?; echo "c5 rc=$rc"; tail -c 1500 $O/c5.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 > $O/c3.log 2>&1; rc=$?; echo "c3 rc=$rc"; tail -c 1500 $O/c3.log
