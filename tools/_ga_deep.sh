# BASELINE config 4 search: S=(3,4,5) kernels (20,50,100) + BatchNorm, RR-GA pop 32, fp32 full protocol,
# checkpointed per generation (resumed from ckpt_seed/ga_deep when present)
CKPT=gpurun_out/ga_deep/ckpt SEED_CKPT=ckpt_seed/ga_deep GENS=${GENS:-12} BUDGET=${BUDGET:-840} TIME=1080 TAG=${TAG:-} \
  GA_ARGS="--space deep --batch-norm" bash tools/gpu.sh ga
