bash tools/gpu_r3_tests.sh && bash tools/gpu_r3_ab.sh && W=decrypt bash tools/gpu_r3_ab.sh
