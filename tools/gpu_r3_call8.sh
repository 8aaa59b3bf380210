#!/bin/bash
bash tools/gpu_r3_bench_all.sh && bash tools/gpu_r3_prof.sh sign && bash tools/gpu_r3_prof.sh dkg --workload dkg
