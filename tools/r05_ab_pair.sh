set -o pipefail
mkdir -p gpurun_out/r05_b
P=$PWD/ntt_amd/libntt_pair.so
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-parity > gpurun_out/r05_b/base_$i.json 2>>gpurun_out/r05_b/err.log || exit 1
  NTT_LIB_PATH=$P timeout -k 10 120 python bench.py --no-cpu-baseline --no-parity > gpurun_out/r05_b/pair_$i.json 2>>gpurun_out/r05_b/err.log || exit 1
done
NTT_LIB_PATH=$P timeout -k 10 400 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_b/pytest_pair.log 2>&1
