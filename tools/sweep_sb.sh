B="python bench.py --steps 5 --warmup 2 --cpu-iters 0"
export APPNP_TUNING=1  # round 6: the library reads tuning overrides only with APPNP_TUNING=1
tools/gpu_session.sh \
 "sb16k::120::APPNP_SB_ROWS=16384 $B" \
 "sb32k::120::APPNP_SB_ROWS=32768 $B" \
 "sb64k::120::APPNP_SB_ROWS=65536 $B" \
 "sb128k::120::APPNP_SB_ROWS=131072 $B" \
 "pmc_l2::200::timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o run --output-format csv -- $B"
