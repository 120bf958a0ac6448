#!/bin/bash
# Round-4: (1) conv_x6sc with paired row groups (two accumulation chains interleaved) against conv_x6s;
# (2) wgrad_x6c with the offsets dealt to the waves per block by chunk count (v7) against the fixed
# o = wave + 8 a (v3, the product form).  A = product library, B = experiments build (-DMSP_SHARED_LISTS=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/3d-weakly-supervised-semantic-segmentation_amd/lib
LEVELS=1,2,3,4 PASSES=fwd,bwd FORMS=local N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04m_A1.log 2>&1 || exit 1
MI3DSPARSE_LIB=$L/libmi3dsparse_exp.so LEVELS=1,2,3,4 PASSES=fwd,bwd FORMS=local,x6s_v2000,x6s_v2400 EXP_VARIANTS=2000,2400 N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04m_B1.log 2>&1 || exit 1
MI3DSPARSE_LIB=$L/libmi3dsparse_exp.so LEVELS=0,1,2,3 PASSES=wgrad WFORMS=chunk,x6c_v3,x6c_v7 WEXP_VARIANTS=3,7 N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04m_W1.log 2>&1 || exit 1
MI3DSPARSE_LIB=$L/libmi3dsparse_exp.so LEVELS=0,1,2,3 PASSES=wgrad WFORMS=chunk,x6c_v3,x6c_v7 WEXP_VARIANTS=7,3 N=20 timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r04m_W2.log 2>&1 || exit 1
cat gpurun_out/kb_r04m_A1.log gpurun_out/kb_r04m_B1.log gpurun_out/kb_r04m_W1.log gpurun_out/kb_r04m_W2.log
