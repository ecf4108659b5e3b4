V=dct-carver_amd/build/variants
bash tools/gpu.sh \
 "tests:-k 'refine or tie_dense or stress or failed_call or dense or config3 or config5 or n16'" \
 "py:tools/fix_study.py --frames lineart,grid8,dots,text --iters 5" \
 "py:tools/fix_study.py --frames lineart_grey,grid8,dots64_grey,text4_grey --iters 5 --lib $V/pg1.so" \
 "py:tools/fix_study.py --frames lineart,grid8,dots,text --iters 5 --lib $V/old.so" \
 "py:tools/fix_study.py --frames lineart,grid8,dots,text --iters 5" \
 "py:tools/fix_study.py --size 8192 --n 16 --frames lineart,dots --iters 5"
