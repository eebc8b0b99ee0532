mkdir -p gpurun_out/r4_skab && timeout -k 10 400 python -u scripts/gemm_skinny_ab.py --ms 64,160 --blocks 256,512 --variants nr8,nt --rounds 3 > gpurun_out/r4_skab/skinny_ab.log 2>&1
