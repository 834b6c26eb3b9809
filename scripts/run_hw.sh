#!/bin/bash
# Test, then package, a homework (the reference's scripts/run_hw.sh): a failed test aborts, a timeout
# still packages (exit status 2 is passed through), as the reference does.
#
#   scripts/run_hw.sh 1 <lastname> <firstname> [test_hw.sh options]
set -u
DIR=$(dirname "$(realpath "$0")")
if [ "$#" -lt 3 ]; then echo "usage: $0 <homework_number> <lastname> <firstname> [test options]"; exit 1; fi
HW=$1 LAST=$2 FIRST=$3
shift 3
echo "==> testing homework $HW"
bash "$DIR/test_hw.sh" "$HW" "$@"
rc=$?
if [ $rc -eq 1 ]; then echo "!!! tests failed: not packaging !!!"; exit 1; fi
[ $rc -eq 2 ] && echo "==> tests inconclusive (timeout): packaging anyway"
echo "==> packaging homework $HW"
bash "$DIR/package_hw.sh" "$HW" "$LAST" "$FIRST" || exit 1
exit $rc
