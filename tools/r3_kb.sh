set -o pipefail
export TMPDIR=/tmp
for pc in 1 2 3; do
echo "== SDPNET_ATTN_PER_CU=$pc"
SDPNET_ATTN_PER_CU=$pc timeout -k 10 120 python -u tools/kern_bench.py --only attn
done
timeout -k 10 120 python -u tools/kern_bench.py --only dw,ln,stats
