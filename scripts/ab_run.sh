mkdir -p gpurun_out/ab1
for v in base rowskip; do
  NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_$v.so REPS=5 timeout -k 10 120 python scripts/dev_scan_timing.py 1024 300 > gpurun_out/ab1/c4_$v.log 2>&1 || exit 1
  NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_$v.so timeout -k 10 120 python scripts/dev_overlap_timing.py c5 8 1 > gpurun_out/ab1/c5_$v.log 2>&1 || exit 1
done
