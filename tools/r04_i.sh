# round-4 call i: CWT two-pass workspace size (Infinity-Cache residency of A) and pass512_two
# at eight waves per SIMD
bash tools/ab_cwt.sh i JW_CWT_GROUP_MB=32 JW_CWT_GROUP_MB=64 && bash tools/ab_cwt_libs.sh i p2w8
