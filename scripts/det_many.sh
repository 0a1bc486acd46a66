#!/bin/bash
# fresh-process repeatability (scripts/det_loop.py): $1 = output dir, $2 = processes per variant,
# then the variants ("-" or NAME=VALUE[,NAME=VALUE])
O=$1; P=$2; shift 2
mkdir -p "$O"
for v in "$@"; do
    for p in $(seq 1 "$P"); do
        if [ "$v" = "-" ]; then
            timeout -k 10 120 python scripts/det_loop.py ${DET_N:-8192} ${DET_Q:-4096} 3 ${DET_DT:-f64} > "$O/det_base_$p.txt" 2>&1 || exit $?
        else
            env $(echo "$v" | tr "," " ") timeout -k 10 120 python scripts/det_loop.py ${DET_N:-8192} ${DET_Q:-4096} 3 ${DET_DT:-f64} > "$O/det_${v//[=,]/_}_$p.txt" 2>&1 || exit $?
        fi
    done
done
grep -H "differ\|rep" "$O"/det_*.txt
