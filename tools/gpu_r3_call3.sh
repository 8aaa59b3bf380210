#!/bin/bash
# round 3 re-entry: whole -m gpu suite + smoke on the rebuilt library, then the WAVE/PAIR crossover
bash tools/gpu_r3_tests.sh && bash tools/gpu_r3_crossover.sh
