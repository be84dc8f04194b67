"""CPU: the Kotlin binding INTEGRATION.md tells a maintainer to add matches the
JNI surface librfa exports.  Every ``external fun`` in the document's Kotlin
blocks is parsed and compared, argument by argument, with the prototype in
include/rfa_jni.h (the JNIEnv* / jobject pair aside) and with the exported
symbol, so a wrong-arity extern in the doc fails here instead of at the first
JNI call."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PREFIX = "Java_com_mantz_1it_nativedsp_NativeDsp_"

KOTLIN_TO_JNI = {"Int": "jint", "Long": "jlong", "Float": "jfloat", "Boolean": "jboolean",
                 "ByteArray": "jbyteArray", "IntArray": "jintArray", "FloatArray": "jfloatArray",
                 "FloatArray?": "jfloatArray", "IntArray?": "jintArray", "ByteArray?": "jbyteArray",
                 None: "void"}


def kotlin_externs():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```kotlin\n(.*?)```", text, flags=re.S)
    out = {}
    for b in blocks:
        b = re.sub(r"//[^\n]*", "", b)
        b = re.sub(r"/\*.*?\*/", "", b, flags=re.S)
        for m in re.finditer(r"external\s+fun\s+(\w+)\s*\((.*?)\)\s*(?::\s*([\w?]+))?", b, flags=re.S):
            name, args, ret = m.group(1), m.group(2), m.group(3)
            types = []
            for a in [x.strip() for x in args.split(",") if x.strip()]:
                pname, ptype = [t.strip() for t in a.split(":")]
                types.append(ptype)
            assert name not in out or out[name] == (types, ret), f"{name} declared twice, differently"
            out[name] = (types, ret)
    return out


def header_prototypes():
    text = open(os.path.join(ROOT, "include", "rfa_jni.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    protos = {}
    for m in re.finditer(r"JNIEXPORT\s+(\w+)\s+JNICALL\s+" + PREFIX + r"(\w+)\s*\((.*?)\)\s*;", text, flags=re.S):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        types = [re.match(r"(.*?)(\w+)$", a.strip()).group(1).replace(" ", "") for a in args.split(",")]
        assert types[:2] == ["JNIEnv*", "jobject"], (name, types[:2])
        protos[name] = (types[2:], ret)
    return protos


def test_doc_externs_match_header():
    doc, hdr = kotlin_externs(), header_prototypes()
    assert len(doc) >= 13, sorted(doc)
    # every native the header declares is shown to the maintainer, and vice versa
    assert sorted(doc) == sorted(hdr), (sorted(set(doc) ^ set(hdr)))
    for name, (types, ret) in doc.items():
        htypes, hret = hdr[name]
        assert [KOTLIN_TO_JNI[t] for t in types] == htypes, (name, types, htypes)
        assert KOTLIN_TO_JNI[ret] == hret, (name, ret, hret)


def test_doc_externs_are_exported():
    import rfanalyzer_amd
    lib = rfanalyzer_amd.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", lib._name], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [PREFIX + n for n in kotlin_externs() if PREFIX + n not in exported]
    assert not missing, missing


@pytest.mark.parametrize("name,arity", [("drawPreprocessNative", 13), ("rowWindowStatsNative", 5),
                                        ("ddcCreate", 5), ("processPacketNative", 5),
                                        ("createAnalyzerNative", 9)])
def test_handle_taking_natives_have_the_handle(name, arity):
    types, _ = kotlin_externs()[name]
    assert len(types) == arity
    if name not in ("ddcCreate", "createAnalyzerNative"):
        assert types[0] == "Long"  # the jlong handle comes first
