AB_TAGS="${HG_TAGS:-base hg}" tools/border_ab.sh || exit 1
LMPC_STAMPS_LIB=tools/build/liblmpc_hgst.so timeout -k 10 200 python -u tools/dense_check.py stamps > gpurun_out/border/st_hg.log 2>&1 || exit 2
grep -E "condense|max cycles" gpurun_out/border/st_hg.log | head -8
