mkdir -p gpurun_out/border
LMPC_STAMPS_OUT=gpurun_out/border/st_border.npz LMPC_STAMPS_LIB=tools/build/liblmpc_stamps.so timeout -k 10 200 python -u tools/dense_check.py stamps > gpurun_out/border/st_border.log 2>&1 || exit 1
LMPC_STAMPS_OUT=gpurun_out/border/st_noborder.npz LMPC_STAMPS_LIB=tools/build/liblmpc_stamps_nb.so timeout -k 10 200 python -u tools/dense_check.py stamps > gpurun_out/border/st_noborder.log 2>&1 || exit 2
grep -A3 "max cycles" gpurun_out/border/st_border.log gpurun_out/border/st_noborder.log
