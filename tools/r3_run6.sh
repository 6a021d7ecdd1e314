set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k flash > gpurun_out/r3_flash.log 2>&1 || { tail -40 gpurun_out/r3_flash.log; exit 1; }
tail -2 gpurun_out/r3_flash.log
timeout -k 10 900 python -u -m pytest tests/test_train.py tests/test_compile.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/r3_train7.log 2>&1 || { tail -40 gpurun_out/r3_train7.log; exit 1; }
tail -2 gpurun_out/r3_train7.log
timeout -k 10 300 python bench.py --config xl_train --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3_xltrain.log 2>&1 || { tail -20 gpurun_out/r3_xltrain.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3_xltrain.log').read().strip().splitlines()[-1]); print('xl_train', d['value'], d['ms_per_step'], d['skipped_steps'], d['loss'], d['peak_mem_gb'])"
for s in 1 2 3; do timeout -k 10 200 python bench.py --no-cpu-baseline --streams $s --steps 60 > gpurun_out/r3_streams_$s.log 2>&1 || exit 1; echo "streams $s $(grep -o "\"value\": [0-9.]*" gpurun_out/r3_streams_$s.log)"; done
