set -o pipefail
timeout -k 10 120 python tools/dbg/epi_dbg.py 2>&1 | grep -v amdgpu.ids
