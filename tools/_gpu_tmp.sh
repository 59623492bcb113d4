set -o pipefail
for args in "8 4 6554 1" "10 4 6554 1" "10 4 6554 2" "8 4 8192 1" "10 4 8192 1" "10 4 8192 2" "10 4 413 1" "10 4 413 2" "8 4 6554 4" "10 4 6554 4"; do
  timeout -k 10 120 python3 tools/_dbg_oop.py $args 4 2>&1 | grep -v amdgpu.ids || exit 1
done
