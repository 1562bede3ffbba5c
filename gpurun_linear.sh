set -u
mkdir -p gpurun_out
( echo v3; timeout -k 10 120 python tools/linear_bench.py --shape 128,32,32 --shape 65536,32,32
  echo v2; MININF_AMD_LINEAR_TUNE=2 timeout -k 10 120 python tools/linear_bench.py --shape 128,32,32 --shape 65536,32,32
  echo valu; timeout -k 10 120 python tools/linear_bench.py --valu --shape 128,32,32 --shape 128,4,32 --shape 65536,32,32 ) > gpurun_out/linear_c4.log 2>&1
