#!/bin/bash
# round-4 measurement bundle: compaction + rollup + tile A/B (r04_e), percentile (r04_f), k_fast PMC (r04_g)
set -o pipefail
bash tools/runs/r04_e.sh ${1:-r04e} && bash tools/runs/r04_f.sh ${2:-r04f} && bash tools/runs/r04_g.sh ${3:-r04g}
