"""Host-code sanitizer runs of the native runtime, CPU only - never on a GPU box.

Builds a second copy of the `_C` extension whose host translation unit (bindings.cpp, which
#includes the C++ runtime: checkpoint engine, gradient-bucket reducer, P2P host side) is
instrumented with AddressSanitizer or ThreadSanitizer (device code untouched: the kernel objects
of the normal build are linked as they are), then runs the CPU checkpoint / trainer tests
against it through RTDC_EXT_SO with the sanitizer runtime preloaded into the (uninstrumented)
interpreter.  Reports only concern our instrumented code; the run fails on the first report.

    python scripts/sanitize_host.py asan|tsan [pytest args...]
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ray_torch_distributed_checkpoint_amd import _build  # noqa: E402

RT = "/opt/rocm/lib/llvm/lib/clang"
TESTS = ["tests/test_checkpoint_format.py", "tests/test_robustness_cpu.py", "tests/test_state_dict_cpu.py",
         "tests/test_dcp_simulate_cpu.py", "tests/test_zero_ckpt_cpu.py"]


def runtime(kind: str) -> str:
    libs = glob.glob(os.path.join(RT, "*", "lib", "linux", f"libclang_rt.{kind}-x86_64.so"))
    if not libs:
        raise SystemExit(f"no {kind} runtime under {RT}")
    return sorted(libs)[-1]


def build(kind: str) -> str:
    _build.build()  # the normal objects (kernels) first
    out_dir = os.path.join("/tmp", f"rtdc_{kind}")
    os.makedirs(out_dir, exist_ok=True)
    tdir, incs, abi = _build._torch_paths()
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flag = "address" if kind == "asan" else "thread"
    bobj = os.path.join(out_dir, "bindings.o")
    cmd = [hipcc, "-O1", "-g", "-fno-omit-frame-pointer", "-Xarch_host", f"-fsanitize={flag}", "-fPIC", "-std=c++17",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-DTORCH_EXTENSION_NAME={_build.EXT_NAME}",
           "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", _build.CSRC]
    for i in incs:
        cmd += ["-I", i]
    cmd += ["-c", os.path.join(_build.CSRC, "bindings.cpp"), "-o", bobj]
    subprocess.run(cmd, check=True)
    kobjs = [o for o in glob.glob(os.path.join(_build.BUILD_DIR, "*.o")) if not o.endswith("bindings.o")]
    so = os.path.join(out_dir, os.path.basename(_build.ext_path()))
    link = [hipcc, "-shared", "-fPIC", f"--offload-arch={_build._arch()}", "-Xarch_host", f"-fsanitize={flag}",
            "-shared-libsan", bobj, *kobjs, "-o", so, "-L", os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch",
            "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lz", f"-Wl,-rpath,{os.path.join(tdir, 'lib')}"]
    subprocess.run(link, check=True)
    return so


def main(argv):
    kind = argv[0] if argv else "asan"
    so = build(kind)
    env = dict(os.environ, RTDC_EXT_SO=so, RTDC_FORCE_CPU="1", PYTHONMALLOC="malloc",
               LD_PRELOAD=runtime(kind))
    if kind == "asan":
        env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:detect_odr_violation=0:protect_shadow_gap=0"
    else:
        # torch's own (uninstrumented) threading - e.g. gloo's AsyncWork teardown - is not ours
        sup = os.path.join("/tmp", "rtdc_tsan", "suppressions.txt")
        with open(sup, "w") as f:
            f.write("race:c10d::\nrace:gloo::\ncalled_from_lib:libtorch_cpu.so\ncalled_from_lib:libtorch_python.so\n"
                    "called_from_lib:libgloo.so\ndeadlock:c10d::\n")
        env["TSAN_OPTIONS"] = (f"halt_on_error=1:report_signal_unsafe=0:second_deadlock_stack=1:suppressions={sup}"
                               ":ignore_noninstrumented_modules=1:report_mutex_bugs=0")
    args = argv[1:] or TESTS
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider", *args],
                       cwd=ROOT, env=env)
    return r.returncode


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
