# A timing build of this tree whose association kernel at the product's narrow widths carries the
# phase timers (EKF_OPT_SCAN_STAMPS: the product launches scan_kernel<T, true, 0> at 192 landmarks
# per workgroup only, and the context then picks 192): slam_ros_amd/lib/xp_stamps128.so, selected
# by SLAM_EKF_LIB. 128-landmark HOT = 2 workgroups with timers; the arithmetic is the product's.
# usage: bash scripts/r06/stamp_build.sh [KERNELS.hip [NAME]]  (default: this tree's, stamps128)
set -e
cd "$(dirname "$0")/../.."
T=$(mktemp -d)
mkdir -p $T/include $T/p/csrc
cp include/slam_ekf.h $T/include/
cp slam_ros_amd/csrc/*.h slam_ros_amd/csrc/ekf_api.hip $T/p/csrc/
cp "${1:-slam_ros_amd/csrc/ekf_kernels.hip}" $T/p/csrc/ekf_kernels.hip
python3 - "$T/p/csrc" <<'PY'
import sys
d = sys.argv[1]
p = d + "/ekf_kernels.hip"; s = open(p).read()
a = "if (p.dbg || precision == EKF_PREC_F64 || p.r_mode == 1 || p.d.kmax != 16) return hipErrorInvalidValue;"
assert a in s; s = s.replace(a, a.replace("p.dbg || ", ""))
b = "        if (half) hipLaunchKernelGGL((scan_kernel<_Float16, false, 2, 128>), grid, block, 0, st, p);\n        else hipLaunchKernelGGL((scan_kernel<float, false, 2, 128>), grid, block, 0, st, p);"
assert b in s
s = s.replace(b, "        if (p.dbg) hipLaunchKernelGGL((scan_kernel<float, true, 2, 128>), grid, block, 0, st, p);\n        else " + b.strip())
open(p, "w").write(s)
p = d + "/ekf_api.hip"; s = open(p).read()
a = "    if (c->dbg || c->sh_world > 0 ||"
assert a in s; s = s.replace(a, "    if (c->sh_world > 0 ||")
open(p, "w").write(s)
PY
python3 -c "import sys; sys.path.insert(0, '.'); from slam_ros_amd import build as b; b.build_variant('slam_ros_amd/lib/xp_${2:-stamps128}.so', [], csrc='$T/p/csrc')"
rm -rf $T
