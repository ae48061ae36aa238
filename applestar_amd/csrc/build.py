"""Build the in-tree native extension ``applestar_amd/_C.<abi>.so`` for gfx950.

* ``csrc/kernels/*.hip`` -> ``hipcc --offload-arch=gfx950 -O3`` (pure HIP, no torch headers: fast)
* ``csrc/bindings.cpp``  -> ``g++`` against the PyTorch-ROCm headers (pybind11 + ATen)
* link with libtorch / c10_hip / amdhip64.

Incremental via ninja (a build.ninja is generated under ``build/csrc``).  No hipify, no CUDA
sources: kernels are written for CDNA4 directly.  Usage: ``python -m applestar_amd.csrc.build``.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
# Build variants: APPLESTAR_BUILD=debug adds -g and device-side bounds asserts (AS_DEBUG);
# APPLESTAR_HOST_SANITIZE=address|undefined|thread instruments the HOST code only (bindings + the host
# halves of the .hip launchers, via -Xarch_host); GPU sanitizers / xnack are not used on this pool.
# APPLESTAR_BUILD=shortpoll: the split-LSTM exchange with the round-2 poll budget of 2^16 passes (diagnostics).
VARIANT = os.environ.get('APPLESTAR_BUILD', 'release')
SANITIZE = os.environ.get('APPLESTAR_HOST_SANITIZE', '')
BUILD = os.path.join(ROOT, 'build', 'csrc' + ('' if VARIANT == 'release' and not SANITIZE else
                                              f'-{VARIANT}{"-" + SANITIZE if SANITIZE else ""}'))
ARCH = os.environ.get('APPLESTAR_OFFLOAD_ARCH', 'gfx950')
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, 'include'), os.path.join(tdir, 'include', 'torch', 'csrc', 'api', 'include')]
    lib = os.path.join(tdir, 'lib')
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def ext_filename() -> str:
    """Release builds land in-tree (what the package imports); debug / sanitizer variants stay in
    their build directory and are loaded with ``APPLESTAR_EXT_PATH=<that .so>``."""
    suffix = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
    if VARIANT == 'release' and not SANITIZE:
        return os.path.join(PKG, '_C' + suffix)
    return os.path.join(BUILD, '_C' + suffix)


def write_ninja() -> str:
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()['include']
    kernels = sorted(glob.glob(os.path.join(HERE, 'kernels', '*.hip')))
    hipcc = os.path.join(ROCM, 'bin', 'hipcc')
    hip_flags = (f'--offload-arch={ARCH} -O3 -fPIC -std=c++17 -fno-gpu-rdc -I{HERE} '
                 f'-D__HIP_PLATFORM_AMD__ -Wno-unused-result')
    if VARIANT == 'debug':
        hip_flags += ' -g -DAS_DEBUG'
    if VARIANT == 'shortpoll':      # diagnostics: the round-2 split-LSTM poll budget (tools/diag/graph_sync_diag.py)
        hip_flags += ' -DAS_SPLIT_POLL_LIMIT=65536u'
    if SANITIZE:
        hip_flags += f' -Xarch_host -fsanitize={SANITIZE}'
    cxx_flags = ' '.join([
        '-O2 -fPIC -std=c++17 -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DTORCH_EXTENSION_NAME=_C',
        '-DTORCH_API_INCLUDE_EXTENSION_H', f'-D_GLIBCXX_USE_CXX11_ABI={abi}', f'-I{HERE}',
        ' '.join(f'-isystem {p}' for p in inc), f'-isystem {py_inc}', f'-isystem {ROCM}/include',
        '-Wno-deprecated-declarations'] + ([f'-fsanitize={SANITIZE} -fno-omit-frame-pointer'] if SANITIZE else [])
        + (['-g -DAS_DEBUG'] if VARIANT == 'debug' else []))
    ldflags = ' '.join([f'-L{lib}', '-lc10', '-ltorch', '-ltorch_cpu', '-ltorch_python', '-lc10_hip', '-ltorch_hip',
                        f'-L{ROCM}/lib', '-lamdhip64', f'-Wl,-rpath,{lib}', f'-Wl,-rpath,{ROCM}/lib']
                       + ([f'-fsanitize={SANITIZE}'] if SANITIZE else []))
    lines = [
        'ninja_required_version = 1.3',
        f'hipcc = {hipcc}',
        f'hipflags = {hip_flags}',
        f'cxxflags = {cxx_flags}',
        f'ldflags = {ldflags}',
        'rule hip',
        '  command = $hipcc $hipflags -c $in -o $out -MD -MF $out.d',
        '  depfile = $out.d',
        '  deps = gcc',
        '  description = HIPCC $in',
        'rule cxx',
        '  command = g++ $cxxflags -c $in -o $out -MD -MF $out.d',
        '  depfile = $out.d',
        '  deps = gcc',
        '  description = CXX $in',
        'rule link',
        '  command = g++ -shared $in -o $out $ldflags',
        '  description = LINK $out',
    ]
    objs = []
    for k in kernels:
        o = os.path.join(BUILD, os.path.basename(k) + '.o')
        lines.append(f'build {o}: hip {k}')
        objs.append(o)
    for cpp in ('bindings.cpp', 'codec.cpp'):
        b_o = os.path.join(BUILD, cpp.replace('.cpp', '.o'))
        lines.append(f'build {b_o}: cxx {os.path.join(HERE, cpp)}')
        objs.append(b_o)
    lines.append(f'build {ext_filename()}: link {" ".join(objs)}')
    lines.append(f'default {ext_filename()}')
    os.makedirs(BUILD, exist_ok=True)
    path = os.path.join(BUILD, 'build.ninja')
    with open(path, 'w') as f:
        f.write('\n'.join(lines) + '\n')
    return path


def host_ext_filename() -> str:
    suffix = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
    if VARIANT == 'release' and not SANITIZE:
        return os.path.join(PKG, '_host' + suffix)
    return os.path.join(BUILD, '_host' + suffix)


def build_host() -> str:
    """Host-only runtime extension (``csrc/host/*.cpp``: shm channels), plain g++ + pybind11, no torch."""
    import pybind11
    out = host_ext_filename()
    srcs = sorted(glob.glob(os.path.join(HERE, 'host', '*.cpp')))
    deps = srcs + sorted(glob.glob(os.path.join(HERE, 'host', '*.h')))
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(s) for s in deps):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    flags = ['-O2', '-shared', '-fPIC', '-std=c++17', '-Wall', '-pthread', f'-I{pybind11.get_include()}',
             f'-I{sysconfig.get_paths()["include"]}']
    if VARIANT == 'debug':
        flags += ['-g', '-O0']
    if SANITIZE:
        flags += [f'-fsanitize={SANITIZE}', '-fno-omit-frame-pointer', '-g']
    subprocess.run(['g++', *flags, *srcs, '-o', out, '-lrt'], check=True)
    return out


def build(verbose: bool = False, jobs: int | None = None) -> str:
    build_host()
    path = write_ninja()
    ninja = shutil.which('ninja')
    if ninja is None:
        import ninja as _ninja  # wheel
        ninja = os.path.join(_ninja.BIN_DIR, 'ninja')
    jobs = jobs or min(8, os.cpu_count() or 4)
    cmd = [ninja, '-f', path, f'-j{jobs}'] + (['-v'] if verbose else [])
    subprocess.run(cmd, check=True, cwd=BUILD)
    return ext_filename()


if __name__ == '__main__':
    out = build(verbose='-v' in sys.argv)
    print(out)
