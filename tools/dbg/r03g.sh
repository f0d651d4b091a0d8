set -o pipefail
bash tools/dbg/r03e.sh; rc=$?; case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/dbg/r03f.sh
