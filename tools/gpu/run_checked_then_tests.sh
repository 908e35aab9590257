#!/bin/bash
# The guard-band suite, then (unless it ended in a fault / abort / time limit) the product suite + smoke.
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu/run_checked.sh
rc=$?
echo "checked suite rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu/run_tests.sh
rc2=$?
echo "product suite rc=$rc2"
[ $rc -eq 0 ] && exit $rc2
exit $rc
