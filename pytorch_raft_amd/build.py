"""Build the in-tree native extension ``pytorch_raft_amd/_C.so`` for gfx950.

    python -m pytorch_raft_amd.build [--force] [-j N]

* every ``csrc/kernels/*.hip`` is compiled by ``hipcc --offload-arch=gfx950 -O3`` WITHOUT torch
  headers (plain HIP, seconds per file);
* ``csrc/bindings.cpp`` (TORCH_LIBRARY registration) is compiled against the installed torch;
* everything is linked into one shared object next to this file, so it travels with the repo
  snapshot to the GPU box and is what ``torch.ops.load_library`` loads at import time.

Incremental: an object is rebuilt when its source or any header in csrc/ is newer.
A second, CPU-only library ``_cpu.so`` (csrc/cpu/*.cpp: image resampling / PNG16 codec used by the
data pipeline) is built with g++ the same way.
"""
import argparse
import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, 'csrc')
BUILD = os.path.join(PKG, '..', 'build', 'raft_amd')
OUT = os.path.join(PKG, '_C.so')
OUT_CPU = os.path.join(PKG, '_cpu.so')
ARCH = os.environ.get('RAFT_AMD_ARCH', 'gfx950')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')


def _torch_paths():
    import torch.utils.cpp_extension as ce
    import torch
    inc = ce.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), 'lib')
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError('command failed (%d):\n%s\n%s' % (r.returncode, ' '.join(cmd), r.stdout))
    return r.stdout


def _up_to_date():
    """Both libraries newer than every source / header: nothing to do (object files not needed,
    so the build/ directory does not have to travel with the tree)."""
    headers = glob.glob(os.path.join(CSRC, '**', '*.h'), recursive=True)
    gpu_srcs = glob.glob(os.path.join(CSRC, 'kernels', '*.hip')) + [os.path.join(CSRC, 'bindings.cpp')]
    cpu_srcs = glob.glob(os.path.join(CSRC, 'cpu', '*.cpp'))
    return not _newer(OUT, gpu_srcs + headers) and not _newer(OUT_CPU, cpu_srcs + headers)


def build(force=False, jobs=None, verbose=False):
    if not force and _up_to_date():
        return OUT
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, '**', '*.h'), recursive=True)
    inc, tlib, abi = _torch_paths()
    jobs = jobs or min(8, os.cpu_count() or 4)

    # ---- GPU extension
    kernels = sorted(glob.glob(os.path.join(CSRC, 'kernels', '*.hip')))
    common = ['-O3', '-fPIC', '-std=c++17', '--offload-arch=%s' % ARCH, '-D__HIP_PLATFORM_AMD__=1',
              '-ffp-contract=fast', '-Wno-unused-result']
    jobs_list = []
    objs = []
    for src in kernels:
        obj = os.path.join(BUILD, os.path.basename(src) + '.o')
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs_list.append([HIPCC] + common + ['-c', src, '-o', obj])
    bsrc = os.path.join(CSRC, 'bindings.cpp')
    bobj = os.path.join(BUILD, 'bindings.o')
    objs.append(bobj)
    if force or _newer(bobj, [bsrc] + headers):
        flags = ['-O2', '-fPIC', '-std=c++17', '-D__HIP_PLATFORM_AMD__=1', '-DUSE_ROCM=1',
                 '-DHIPBLAS_V2', '-D_GLIBCXX_USE_CXX11_ABI=%d' % abi, '-Wno-unused-result',
                 '-Wno-deprecated-declarations']
        flags += ['-I' + p for p in inc]
        jobs_list.append([HIPCC] + flags + ['-c', bsrc, '-o', bobj])

    # ---- CPU helper library (data pipeline)
    cpu_srcs = sorted(f for f in glob.glob(os.path.join(CSRC, 'cpu', '*.cpp'))
                      if not f.endswith('sanitize_main.cpp'))
    cpu_objs = []
    for src in cpu_srcs:
        obj = os.path.join(BUILD, 'cpu_' + os.path.basename(src) + '.o')
        cpu_objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs_list.append(['g++', '-O3', '-fPIC', '-std=c++17', '-march=x86-64-v2', '-fopenmp',
                              '-c', src, '-o', obj])

    if jobs_list:
        with ThreadPoolExecutor(max_workers=jobs) as ex:
            for out in ex.map(_run, jobs_list):
                if verbose and out.strip():
                    print(out)

    if force or _newer(OUT, objs):
        link = [HIPCC, '-shared', '-fPIC', '--offload-arch=%s' % ARCH] + objs + [
            '-L' + tlib, '-lc10', '-lc10_hip', '-ltorch', '-ltorch_cpu', '-ltorch_hip',
            '-Wl,-rpath,' + tlib, '-o', OUT + '.tmp']
        _run(link)
        os.replace(OUT + '.tmp', OUT)
    if cpu_objs and (force or _newer(OUT_CPU, cpu_objs)):
        _run(['g++', '-shared', '-fPIC', '-fopenmp'] + cpu_objs + ['-o', OUT_CPU + '.tmp'])
        os.replace(OUT_CPU + '.tmp', OUT_CPU)
    return OUT


SANITIZE_FLAGS = ['-fsanitize=address,undefined,float-cast-overflow', '-fno-sanitize-recover=all',
                  '-fno-omit-frame-pointer', '-g', '-O1', '-std=c++17']


def build_sanitized(run=True):
    """Host-code sanitizer build: csrc/cpu/*.cpp + the csrc/cpu/sanitize_main.cpp driver linked into
    one ASan/UBSan executable (no GPU code involved), optionally run.  Returns (path, output)."""
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, 'cpu', '*.cpp')))
    exe = os.path.join(BUILD, 'imgproc_sanitize')
    if _newer(exe, srcs + glob.glob(os.path.join(CSRC, 'cpu', '*.h'))):
        _run(['g++'] + SANITIZE_FLAGS + srcs + ['-o', exe])
    out = ''
    if run:
        env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0',
                   UBSAN_OPTIONS='print_stacktrace=1')
        r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
        out = r.stdout
        if r.returncode != 0:
            raise RuntimeError('sanitizer run failed (%d):\n%s' % (r.returncode, out))
    return exe, out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--force', action='store_true')
    ap.add_argument('-j', type=int, default=None)
    ap.add_argument('-v', action='store_true')
    ap.add_argument('--sanitize', action='store_true',
                    help='build + run the ASan/UBSan executable of the CPU image runtime')
    a = ap.parse_args(argv)
    if a.sanitize:
        exe, out = build_sanitized()
        print(out.strip())
        return
    out = build(force=a.force, jobs=a.j, verbose=a.v)
    print('built', out)


if __name__ == '__main__':
    main()
