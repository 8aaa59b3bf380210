#!/bin/bash
set -o pipefail
./tools/gpu_r2_prof.sh sign && ./tools/gpu_r2_prof.sh decrypt --workload decrypt && ./tools/gpu_r2_prof.sh dkg --workload dkg && python3 tools/pmc_traffic.py gpurun_out/prof/pmc_traffic.json gpurun_out/prof/sign gpurun_out/prof/decrypt gpurun_out/prof/dkg
