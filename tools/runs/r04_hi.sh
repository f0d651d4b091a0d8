#!/bin/bash
set -o pipefail
bash tools/runs/r04_h.sh && bash tools/runs/r04_i.sh
