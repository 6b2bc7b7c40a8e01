# Register / scratch usage of a library's kernels: bash scripts/kres.sh [lib.so] [name-regex]
set -e
LIB=$(readlink -f ${1:-slam_ros_amd/lib/libslam_ekf.so})
PAT=${2:-scan_kernel}
T=$(mktemp -d)
cp $LIB $T/lib.so
(cd $T && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading lib.so > /dev/null)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/lib.so.0.hipv4-amdgcn-amd-amdhsa--gfx950 | \
  python3 -c "
import sys, re
pat = re.compile(sys.argv[1]); cur = {}; out = []
for line in sys.stdin:
    m = re.match(r'\s*-?\s*\.(\w+):\s+(.*)', line)
    if not m: continue
    k, v = m.groups()
    if k == 'args': cur = {}
    cur[k] = v
    if k == 'vgpr_spill_count':
        out.append(dict(cur))
for d in out:
    if pat.search(d.get('name', '')):
        print(d.get('name'), 'lds', d.get('group_segment_fixed_size'), 'vgpr', d.get('vgpr_count'), 'agpr', d.get('agpr_count'), 'sgpr_spill', d.get('sgpr_spill_count'), 'vgpr_spill', d.get('vgpr_spill_count'), 'scratch', d.get('private_segment_fixed_size'))
" "$PAT"
rm -rf $T
