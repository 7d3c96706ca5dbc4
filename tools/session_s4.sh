F="--cpu-seconds 0.3 --no-latency --no-kernel-timing"
PYTEST_SECS=400 bash tools/gpu.sh r05_s4 tests="tests/test_gpu_sysor.py tests/test_gpu_parity.py::test_batch_equals_singles" \
 bench_B1="--cpu-seconds 0 --option sysor=1" bench_D1="--config D --cpu-seconds 0 --option sysor=1" \
 bench_p0="$F" bench_p2="$F --chunk 1024 --option pipeline=2" \
 bench_p2s2="$F --chunk 1024 --option pipeline=2 --option split_cus=2" \
 bench_p2s2c6="$F --chunk 1024 --option pipeline=2 --option split_cus=2 --option chain_cus=6" \
 bench_p2s1c7="$F --chunk 1024 --option pipeline=2 --option split_cus=1 --option chain_cus=7" \
 bench_p2s3c5="$F --chunk 1024 --option pipeline=2 --option split_cus=3 --option chain_cus=5" \
 bench_p1s2c6="$F --chunk 512 --option pipeline=1 --option split_cus=2 --option chain_cus=6" \
 bench_p2s2c6b="$F --chunk 512 --option pipeline=2 --option split_cus=2 --option chain_cus=6"
