#!/bin/bash
# run every built phase_micro_* variant once (GPU box), each time-limited
cd "$(dirname "$0")"
for b in phase_micro_*; do
  [ -x "$b" ] || continue
  echo -n "$b: "; timeout -k 10 60 ./$b || exit 1
done
