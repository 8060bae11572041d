#!/bin/bash
# GPU check run: focused tests, then benches + a kernel profile. A test failure does not stop the
# benches; a crash / timeout / abort (124, 134, 137, 139) stops everything after it.
OUT=${OUT:-gpurun_out/check}
mkdir -p "$OUT"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -3 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
for step in "$@"; do
  eval "$step" || exit $?
done
