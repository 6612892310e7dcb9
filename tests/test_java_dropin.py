"""The Java drop-in at the reference's result-collect call sites.

LogisticRegression.scala:290-291 casts its store to DoubleArrayStore and
Word2Vec.scala:814-817 to FloatMatrixStoreAdaGrad, then iterate them. So a GPU
store must BE the concrete class: integration/jni/Gpu<Store>.java extends <Store>
for all seven stores of DataStore.createStore (DataStore.java:50-92), overrides every
public method the parent declares (names from tests/golden/ref_store_methods.json;
indexOf / keyOf only read localRows, which init() sets, and stay inherited), and
fills the parent's localData (and AdaGrad's alpha / delta) from the device in
snapshot(), which iter() calls. GpuStores.createStore mirrors the dispatch. No JDK
exists here, so these are source checks; the snapshot entry point itself runs on the
mock JVM on the GPU (tests/test_jni_shim.py::test_mock_jvm_snapshot_on_gpu).
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "integration", "jni")
FIX = os.path.join(ROOT, "tests", "golden", "ref_store_methods.json")
INHERITED = {"indexOf", "keyOf"}  # read localRows only (set by init), no localData


def _src(name):
    return open(os.path.join(JNI, name + ".java")).read()


def _declared(src):
    return set(re.findall(r"^    public (?!class\b|static\b)(?:[\w\[\]<>.]+ )?(\w+)\(", src, re.M))


def test_store_methods_fixture_current():
    if not os.path.isdir("/root/reference"):
        return
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_ref_store_methods
    assert make_ref_store_methods.methods() == json.load(open(FIX))


def test_every_store_has_a_gpu_subclass_overriding_its_methods():
    ref = json.load(open(FIX))
    assert len(ref) == 7
    for parent, methods in ref.items():
        src = _src("Gpu" + parent)
        assert re.search(rf"public class Gpu{parent} extends {parent} \{{", src), parent
        missing = set(methods) - INHERITED - _declared(src)
        assert not missing, (parent, missing)
        # the heap arrays are never allocated at init: only snapshot() fills them
        init = src[src.index("public void init("):]
        init = init[:init.index("\n    }\n")]
        assert "new " in init and "localData" not in init.split("new GpuDataStore")[1], parent
        assert "localData = new" in src and "gpu.snapshot(0," in src
        if "iter" in methods:
            it = src[src.index("public Iter iter()"):]
            assert it.index("snapshot();") < it.index("return super.iter();"), parent
        if parent == "FloatMatrixStoreAdaGrad":
            # Iter.value() prints delta[p] and alpha[p] (:328-331): both filled
            assert "gpu.snapshot(1," in src and "gpu.snapshot(2," in src
            # the per-push report of :246, from the device's maxDelta
            push = src[src.index("public void handlePush("):]
            push = push[:push.index("\n    }\n")]
            assert "gpu.maxDelta(" in push and '"max delta: " + maxDeltaRow + ", " + maxDeltaCol + ", " + maxDelta' in push


def test_factory_mirrors_create_store():
    src = _src("GpuStores")
    made = re.findall(r"(Gpu\w+Store\w*) store = new \1\(format, device\);", src)
    assert sorted(made) == sorted("Gpu" + p for p in json.load(open(FIX))), made
    assert "throw new IllegalArgumentException(\"Unrecognized matrix type: \"" in src


def test_snapshot_natives_declared_and_bound():
    java = _src("GpuDataStore")
    cc = open(os.path.join(JNI, "dml_jni.cc")).read()
    for n in ("nativeSnapshot", "nativeMaxDelta"):
        assert re.search(rf"static native \w+ {n}\(", java), n
        assert f"FN({n})" in cc, n
    assert "dml_store_read_rows" in cc and "dml_store_max_delta" in cc
