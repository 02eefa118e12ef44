set -o pipefail
bash profiles/run_profile.sh r01g_c2 &&
bash profiles/run_profile.sh r01g_c3 --config c3
echo rc=$?
