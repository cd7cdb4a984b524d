cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export LMI_LIB_NAME=liblmi_hip_abl.so
timeout -k 10 300 python -u tools/prof_scan.py --no-subcluster --abl 0,33 > gpurun_out/ck8192.log 2>&1 &&
timeout -k 10 300 python -u tools/prof_scan.py --no-subcluster --abl 0 --chunk-rows 4096 > gpurun_out/ck4096.log 2>&1 &&
timeout -k 10 300 python -u tools/prof_scan.py --no-subcluster --abl 0 --chunk-rows 2048 > gpurun_out/ck2048.log 2>&1 &&
timeout -k 10 300 python -u tools/prof_scan.py --no-subcluster --abl 0 --chunk-rows 16384 > gpurun_out/ck16384.log 2>&1
