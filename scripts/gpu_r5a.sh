set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_lru_stamps.py tests/test_key_shadow.py tests/test_lru_golden.py > gpurun_out/r5a/pytest.log 2>&1 || { tail -30 gpurun_out/r5a/pytest.log; exit 1; }
tail -3 gpurun_out/r5a/pytest.log
timeout -k 10 400 python bench.py > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err || { tail -20 gpurun_out/r5a/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r5a/bench.json')); print(d['value'], d['roofline']['frac'], d['c5']['avg_kernel_ms'], d['verified'])"
