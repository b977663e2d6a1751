set -euo pipefail
mkdir -p gpurun_out/wh
timeout -k 10 300 python3 -u -m pytest tests/test_bvh_tracer.py tests/test_c1_spheres.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wh/pytest.log 2>&1 || { tail -30 gpurun_out/wh/pytest.log; exit 1; }
tail -1 gpurun_out/wh/pytest.log
timeout -k 10 300 python3 tools/ab_libs.py librt_hip_wh0.so librt_hip_fg1.so librt_hip.so librt_hip_fg4s12.so --scene c3 --width 1280 --height 960 --spp 64 --rounds 5 > gpurun_out/wh/ab.json 2>&1
cat gpurun_out/wh/ab.json
