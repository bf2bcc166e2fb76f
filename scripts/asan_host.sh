#!/bin/bash
# Host-code sanitizer runs. First the object formats (csrc/kad_objects.cpp: JSON parser, Go decoders, object edit):
# an ASan + UBSan build of that file alone (no HIP in it), driven by tests/test_native_objects.py's seeded
# parity batches and malformed inputs through the same Python bindings. CPU only.
set -e
cd "$(dirname "$0")/.."
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fPIC -shared -pthread \
    kubeadmiral_amd/csrc/kad_objects.cpp -o /tmp/libkad_objects_asan.so
cat > /tmp/kad_asan_run.py <<'PY'
import ctypes, random, sys
sys.path[:0] = [".", "tests"]
from kubeadmiral_amd import runtime
runtime._lib = ctypes.CDLL("/tmp/libkad_objects_asan.so")  # the bindings below only call kad_units_* / kad_applied_* / kad_trigger_*
import test_native_objects as t
from kubeadmiral_amd import columns as K
for seed in range(1, 6):
    rng = random.Random(seed)
    policies = [t._policy(rng, f"p{i}", i % 2 == 0) for i in range(6)]
    objs = [t._object(rng, policies) for _ in range(400)]
    t.assert_same(t.DEPLOY, objs, policies, threads=4)
    off, cl, rep = t._results(rng, len(objs))
    t.assert_apply_same(t.DEPLOY, objs, off, cl, rep, [True] * len(objs), [None] * len(objs), threads=4)
    K.trigger_prefixes(t.DEPLOY, objs, policies, threads=4)
    K.apply_results_ex(t.DEPLOY, objs, t.NAMES, off, cl, rep, trigger=[str(i) for i in range(len(objs))],
                       ann_only=[i % 3 == 0 for i in range(len(objs))], threads=4)
t.test_trigger_prefixes_match_python()
t.test_apply_with_trigger_annotation_matches_python()
bad = [b"", b"{", b"[", b'{"a":', b'"\\ud800', b"1e400", b'{"x": ' + b"[" * 2000 + b"]" * 2000 + b"}", b"\xff\xfe"]
K.units_from_objects(t.DEPLOY, bad, [{"metadata": {"name": "p"}, "spec": {}}], threads=2)
K.apply_results(t.DEPLOY, bad, t.NAMES, list(range(len(bad) + 1)), [0] * len(bad), [1] * len(bad))
K.trigger_prefixes(t.DEPLOY, bad, [{"metadata": {"name": "p"}, "spec": {}}], threads=2)
K.apply_results_ex(t.DEPLOY, bad, t.NAMES, list(range(len(bad) + 1)), [0] * len(bad), [1] * len(bad),
                   trigger=["1"] * len(bad), ann_only=[i % 2 == 0 for i in range(len(bad))])
print("sanitizers: clean")
PY
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" ASAN_OPTIONS=detect_leaks=0 \
    UBSAN_OPTIONS=halt_on_error=1 python /tmp/kad_asan_run.py

# and the whole library's host code (packer, upload checks, object formats) in an ASan build of libkad.so
# (device code unchanged: -Xarch_host), under the CPU tests of the packer and the object formats
python -c "from kubeadmiral_amd import build; build.build(force=True, out='/tmp/libkad_asan.so', extra=['-Xarch_host', '-fsanitize=address', '-Xarch_host', '-fno-omit-frame-pointer', '-shared-libasan'])"
cat > /tmp/kad_asanplug.py <<'PY'
from kubeadmiral_amd import runtime
runtime._lib = None
runtime.load_library("/tmp/libkad_asan.so")  # every later load_library() returns it
PY
PYTHONPATH=/tmp:. LD_PRELOAD="$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so)" \
    ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0 \
    python -m pytest -p kad_asanplug tests/test_native_pack.py tests/test_native_objects.py -x -q -p no:cacheprovider
