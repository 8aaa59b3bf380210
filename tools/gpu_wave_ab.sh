set -o pipefail
mkdir -p gpurun_out
for v in 1 2 4; do HBBFT_HIP_LIB=$PWD/hbbft_amd/ab/lib_nacc$v.so timeout -k 10 120 python -u tools/wave_ab.py >> gpurun_out/wave_ab.log 2>&1 || exit 1; done
cat gpurun_out/wave_ab.log
