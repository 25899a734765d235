# round-4 call q: ring rotation on (product) vs off (rot0), three alternating reps, 10 steps
REPS="1 2 3" STEPS=10 bash tools/ab_modwt_libs.sh q rot0
