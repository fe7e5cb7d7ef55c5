#!/bin/bash
# A/B of the Python orchestration: the in-tree package vs a copy of HEAD in _ab_base/ (same native modules), each
# config timed twice in alternation with many steps. usage: bash scripts/ab_steps.sh "<bench args>" ...
set -o pipefail
for args in "$@"; do
    for rep in 1 2; do
        for side in base new; do
            if [ $side = base ]; then d=_ab_base; else d=.; fi
            v=$(cd $d && timeout -k 10 300 python bench.py $args 2>/dev/null | grep -o '"ms_per_step": [0-9.]*' | awk '{print $2}') || exit 1
            echo "$args | $side | $v ms/step"
        done
    done
done
