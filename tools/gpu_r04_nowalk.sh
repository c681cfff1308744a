set -o pipefail
TESTS="" bash tools/gpu_ab_env.sh nowalk "FRT_JIT_DBG_NOWALK=0" "FRT_JIT_DBG_NOWALK=1" "FRT_JIT_DBG_NOWALK=2"
