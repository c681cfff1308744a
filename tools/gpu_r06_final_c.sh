#!/bin/bash
# round 6 final evidence (c): the whole -m gpu suite, smoke(), the default bench line (tools/gpu_full.sh), then the
# cfg3 / cfg4 bench lines
set -o pipefail
bash tools/gpu_full.sh r06 || exit 1
bash tools/gpu_r06_cfgs.sh || exit 1
