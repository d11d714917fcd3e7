OUT=gpurun_out/ab5; mkdir -p $OUT
for v in k64 k8 k4; do
  NUSIPROP_LIB=$PWD/nusiprop_amd/libnusi_$v.so timeout -k 10 120 python scripts/dev_cascade_kinds.py 1024 300 > $OUT/kinds_$v.log 2>&1 || exit 1
done
