cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g3
timeout -k 10 300 python bench.py --gpus 2 --same-device --dist-backend gloo --steps 20 --warmup 10 > gpurun_out/g3/out.log 2> gpurun_out/g3/err.log
echo rc=$?
grep -v "amdgpu.ids\|socket.cpp" gpurun_out/g3/err.log | head -60
