mkdir -p gpurun_out
for e in 0 1; do RP_SIM_EARLY=$e timeout -k 10 300 python3 bench.py --no-merge --no-wire --no-cpu --no-api --steps 2 --warmup 1 --batch-log2 20 > gpurun_out/sim_early$e.json 2> gpurun_out/sim_early$e.err; echo "sim early=$e rc=$?"; done
