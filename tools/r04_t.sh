# round-4 call t: CWT knob sweep on the final kernels (workspace size, band threshold, NT stores)
bash tools/ab_cwt.sh t JW_CWT_GROUP_MB=256 JW_CWT_GROUP_MB=512 JW_CWT_BAND=28 JW_CWT_BAND=36 JW_CWT_NT=0 JW_CWT_NT=3
