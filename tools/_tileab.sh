L=dct-carver_amd/build/libdctenergy_hip.so
K="timeout -k 10 120 python tools/kbench.py --rounds 7"
( $K --n 8 --size 4096 --tile-h 0,128,64,32 $L
  $K --n 8 --width 6000 --height 4000 --tile-h 0,128,64 $L
  $K --n 8 --size 2048 --tile-h 0,128,32 $L
  $K --n 8 --size 16384 --tile-h 0,64 $L
  $K --n 16 --size 4096 --tile-h 0,128,64 $L
  $K --exact --n 8 --size 4096 --tile-h 0,64 $L
  $K --exact --n 8 --width 6000 --height 4000 --tile-h 0,128 $L
) 2>&1 | grep -v amdgpu.ids
