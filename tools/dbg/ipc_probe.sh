#!/bin/bash
# two processes: export / import an IPC handle of several sizes, each step timed
cd "${GRAFT_REPO_ROOT:-.}"
for spec in "2416 n 0" "2416 r 0" "2416 r 20" "9 r 0"; do
  set -- $spec; mb=$1; reg=$2; extra=$3
  f=/tmp/ipc_probe_$mb; rm -f $f $f.done
  timeout -k 5 40 ./tools/dbg/ipc_probe 0 $mb $f $reg $extra & a=$!
  timeout -k 5 40 ./tools/dbg/ipc_probe 1 $mb $f $reg $extra & b=$!
  wait $a; ra=$?; wait $b; rb=$?
  echo "size $mb MiB reg $reg extra $extra: rc $ra $rb"
done
exit 0
