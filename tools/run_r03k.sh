R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/kbench.py --variants l12,l12+DM_MFQ_NWMAX=2,l12+DM_MFQ_NWMAX=2+DM_MFQ_MINW=8 --rounds 3 > gpurun_out/r03k_c3_nw.txt 2>&1 && \
timeout -k 10 300 python3 tools/kbench.py --variants l12,l12+DM_MFQ_NWMAX=4 --rounds 2 --tile 256 --grid 16 > gpurun_out/r03k_c5_nw.txt 2>&1
