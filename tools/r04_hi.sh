#!/bin/bash
set -o pipefail
bash tools/r04_h.sh && bash tools/r04_i.sh
