# kernel trace of the emulated N=8 ranks (fused Cornell): where the per-step time goes
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/trace8
RT_EMU_FUSED=1 RT_EMU_STEPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/trace8/raw -o run -- python3 scripts/rank_emulation.py 1 8 > gpurun_out/trace8/emu.txt 2>&1 || exit 1
find gpurun_out/trace8/raw -name "*.csv" | head -20
