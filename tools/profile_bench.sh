#!/bin/bash
# rocprofv3 kernel-trace summary + PMC passes of the N=1 bench (writes under $1).
set -e
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --no-cpu-baseline "$@" > $OUT/kt.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py --no-cpu-baseline "$@" > $OUT/fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --no-cpu-baseline "$@" > $OUT/write.log 2>&1
echo PROFILE_DONE
