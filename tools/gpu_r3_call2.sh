bash tools/gpu_r3_tests.sh tests/test_gpu_wire_msgs.py tests/test_gpu_honey_badger.py tests/test_bench_launch.py && bash tools/gpu_r3_crossover.sh
