"""The JNI shim (integration/jni/dml_jni.cc) compiles: there is no JDK in this image,
so it is checked with g++ -fsyntax-only against tests/jni_stub/jni.h (the JNI
types and JNIEnv members it uses, JNI-spec signatures) and the real
include/distml_ps.h. Also: the shim's native methods are the ones
GpuDataStore.java / GpuShardGroup.java declare, and nativePush copies the
byte[] (GetByteArrayRegion) instead of holding a critical section across the
GPU apply."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "integration", "jni")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_shim_compiles():
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror",
                        "-I", os.path.join(ROOT, "tests", "jni_stub"), "-I", os.path.join(ROOT, "include"),
                        os.path.join(JNI, "dml_jni.cc")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_native_methods_match():
    cc = open(os.path.join(JNI, "dml_jni.cc")).read()
    for cls, macro in (("GpuDataStore", "FN"), ("GpuShardGroup", "GFN")):
        java = open(os.path.join(JNI, cls + ".java")).read()
        declared = set(re.findall(r"native\s+[\w.\[\]]+\s+(\w+)\s*\(", java))
        defined = set(re.findall(r"\b" + macro + r"\((\w+)\)", cc)) - {"name"}  # the macro definitions
        assert declared == defined, (cls, declared ^ defined)


def test_push_does_not_pin_across_the_apply():
    cc = open(os.path.join(JNI, "dml_jni.cc")).read()
    assert "GetPrimitiveArrayCritical" not in cc
