#!/bin/bash
# round-5 PMC of the exact kernels (fp64 op counts per pixel)
L="$GRAFT_REPO_ROOT/dct-carver_amd/build/libdctenergy_hip.so"
exec bash tools/gpu.sh \
  "ppmc:SQ_INSTS_VALU,SQ_WAVES,GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES:tools/kbench.py --exact --n 8 --size 16384 --rounds 1 --iters 2 $L" \
  "ppmc:SQ_INSTS_VALU,SQ_WAVES,GRBM_GUI_ACTIVE,SQ_WAVE_CYCLES:tools/kbench.py --exact --n 16 --size 8192 --rounds 1 --iters 2 $L" \
  "ppmc:SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_TRANS_F64:tools/kbench.py --exact --n 8 --size 16384 --rounds 1 --iters 2 $L"
