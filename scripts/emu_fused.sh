set -u
mkdir -p gpurun_out/final
RT_EMU_FUSED=1 timeout -k 10 300 python scripts/rank_emulation.py > gpurun_out/final/rank_emulation_fused_cornell.log 2>&1 || exit 1
RT_EMU_FUSED=1 RT_EMU_SCENE=bunny timeout -k 10 400 python scripts/rank_emulation.py > gpurun_out/final/rank_emulation_fused_bunny.log 2>&1 || exit 1
cat gpurun_out/final/rank_emulation_fused_*.log
