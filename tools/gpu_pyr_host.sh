set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out/pyr
timeout -k 10 200 python3 tools/host_profile.py 513 pyramid_kv '{"base_size": 512}' > gpurun_out/pyr/host.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
HOST_PROFILE_CALLS=100 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pyr/prof" -o run -- python3 "$R/tools/host_profile.py" 513 pyramid_kv '{"base_size": 512}' > "$R/gpurun_out/pyr/prof.log" 2>&1 || exit 1
