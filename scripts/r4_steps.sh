#!/bin/bash
# Runs each argument as a step (bash -c).  A step that ends 0 or 1 (passed / tests failed)
# lets the next one run; any other status (a time limit, an abort, a crash) ends the script.
set -u
for cmd in "$@"; do
  echo "== step: $cmd"
  bash -c "$cmd"
  rc=$?
  echo "== rc $rc"
  case $rc in
    0|1) ;;
    *) echo "== stopping after rc $rc"; exit $rc ;;
  esac
done
