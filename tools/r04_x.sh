# round-4 call x: SQ counter passes for the cfg5 and headline MODWT kernels and the AUTO kernels
bash tools/pmc_sq.sh cfg5 bench.py --wavelet Symlet8 --levels 6 --steps 1 --warmup 1 --no-alt --no-cpu-baseline --no-check && \
bash tools/pmc_sq.sh cfg2 bench.py --steps 1 --warmup 1 --no-alt --no-cpu-baseline --no-check && \
bash tools/pmc_sq.sh auto tools/modwt_time.py --method auto --arith strict --batch 32 --reps 1
