# M forward bench over the number of sub-batch streams in the graph, interleaved.  Repo root, GPU box.
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for ns in 2 3 4; do
    timeout -k 10 240 python bench.py --streams $ns --no-cpu-baseline > gpurun_out/ns_$ns.log 2>&1 \
      || { tail -20 gpurun_out/ns_$ns.log; exit 1; }
    echo "streams=$ns $(tail -n 1 gpurun_out/ns_$ns.log | grep -o '"value": [0-9.]*')"
  done
done
