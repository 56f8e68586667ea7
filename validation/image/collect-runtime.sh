#!/usr/bin/env bash
# Copy amdgpu-validate plus the shared-library closure it needs at run time
# into DEST (DEST/bin, DEST/lib), so the runtime image is a plain Ubuntu base
# + this directory: no ROCm SDK, compilers or math libraries (hipBLASLt,
# rocBLAS, MIOpen are not linked - the GEMM is our own kernel), which keeps
# the image small and its pull time out of time-to-GPU-ready.
#
# The closure is ldd's (DT_NEEDED, recursive) minus the glibc/libstdc++ family
# the base image already provides, plus the libraries the HIP/HSA runtimes
# dlopen() at run time (those never show up in ldd).
#
# usage: collect-runtime.sh BINARY DEST [ROCM_LIB_DIR]
set -euo pipefail
bin=$1
dest=$2
rocm_lib=${3:-/opt/rocm/lib}
mkdir -p "$dest/bin" "$dest/lib"
cp -L "$bin" "$dest/bin/"

is_base() {  # provided by any glibc-based distro image
  case "$(basename "$1")" in
    libc.so.*|libm.so.*|libdl.so.*|libpthread.so.*|librt.so.*|ld-linux*|libstdc++.so.*|libgcc_s.so.*|linux-vdso*) return 0 ;;
  esac
  return 1
}

copy_closure() {
  ldd "$1" | awk '/=> \// {print $3}' | while read -r lib; do
    is_base "$lib" && continue
    name=$(basename "$lib")
    [ -e "$dest/lib/$name" ] && continue
    cp -L "$lib" "$dest/lib/$name"
  done
}

copy_closure "$bin"
# dlopen()ed by libamdhip64 / libhsa-runtime64 / librccl (code-object and
# device-library handling, optional SMI); copied with their own closures
for opt in libamd_comgr.so.3 libamd_comgr.so.2 libhsa-amd-aqlprofile64.so.1 librocm-core.so.1; do
  if [ -e "$rocm_lib/$opt" ]; then
    cp -L "$rocm_lib/$opt" "$dest/lib/$opt"
    copy_closure "$rocm_lib/$opt"
  fi
done
# runtimes also dlopen() by unversioned name (libhsa-amd-aqlprofile64.so)
for f in "$dest"/lib/*.so.*; do
  base=$(basename "$f")
  unv=${base%%.so.*}.so
  [ -e "$dest/lib/$unv" ] || ln -s "$base" "$dest/lib/$unv"
done
# the image only runs on MI355X: cut every copied library's HIP fat binary to
# gfx950 (librccl.so: 13 targets, 570 MB -> a 66 MB compressed gfx950 bundle in
# place; the gzip'd closure drops from 649 to 150 MB and RCCL's first set-up no
# longer decompresses the other 12 targets: profiles/r5_fatbin). Set
# NTM_KEEP_FATBIN=1 to keep the vendor bundles as they are.
here=$(cd "$(dirname "$0")" && pwd)
if [ "${NTM_KEEP_FATBIN:-0}" != 1 ] && ! command -v python3 > /dev/null; then
  echo "collect-runtime: no python3 in the build image; vendor fat binaries kept whole" >&2
elif [ "${NTM_KEEP_FATBIN:-0}" != 1 ]; then
  for f in "$dest"/lib/*.so.*; do
    [ -L "$f" ] && continue
    python3 "$here/strip-fatbin.py" "$f" --bundler "$rocm_lib/llvm/bin/clang-offload-bundler"
  done
fi
# sanity: nothing unresolved when only DEST/lib is on the search path
if LD_LIBRARY_PATH="$dest/lib" ldd "$dest/bin/$(basename "$bin")" | grep -q "not found"; then
  echo "unresolved libraries:" >&2
  LD_LIBRARY_PATH="$dest/lib" ldd "$dest/bin/$(basename "$bin")" | grep "not found" >&2
  exit 1
fi
du -sh "$dest" | awk '{print "runtime closure: " $1}'
