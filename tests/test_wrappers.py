"""R and Java component wrappers (reference wrappers/s2i/R/
microservice.R:129-304, wrappers/s2i/java/s2i/bin/run).  Neither runtime
exists in this image, so parity with the reference is unpinned; these tests
pin statically what the engine relies on: the internal REST routes per node
type (the paths csrc/server/remote_unit.cc calls), the typed-parameter
rules, the s2i entry points and the builder's contexts."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R_FILE = os.path.join(ROOT, "wrappers", "R", "microservice.R")
JAVA_DIR = os.path.join(ROOT, "wrappers", "java", "src", "main", "java", "io", "seldon", "amd", "wrapper")

# what the engine's remote node client calls per node type (remote_unit.cc)
EXPECTED = {"MODEL": {"/predict", "/send-feedback"}, "ROUTER": {"/route", "/send-feedback"},
            "TRANSFORMER": {"/transform-input", "/transform-output"},
            "OUTPUT_TRANSFORMER": {"/transform-input", "/transform-output"}, "COMBINER": {"/aggregate"}}


def _read(p):
    with open(p) as f:
        return f.read()


def test_engine_client_paths_are_the_wrapper_paths():
    src = _read(os.path.join(ROOT, "csrc", "server", "remote_unit.cc"))
    called = set(re.findall(r'call_(?:message|rest)\("([a-z-]+)"', src))
    assert {p.strip("/") for ps in EXPECTED.values() for p in ps} <= called | {"route", "aggregate",
                                                                               "transform-output"}


def test_r_wrapper_routes_and_rules():
    src = _read(R_FILE)
    block = src[src.index("ROUTES <- list("):src.index(")\n\ndispatch")]
    routes = {m.group(1): set(re.findall(r'"(/[a-z-]+)"', m.group(2)))
              for m in re.finditer(r'(\w+) = c\(([^)]*)\)', block)}
    assert routes == EXPECTED
    for path in {p for ps in EXPECTED.values() for p in ps}:
        assert f'"{path}" = handle_' in src, path
    for t in ("INT = as.integer", "FLOAT = as.numeric", "DOUBLE = as.numeric", "BOOL ="):
        assert t in src, t
    assert 'form_field(body, "json")' in src and 'form_field(req$QUERY_STRING, "json")' in src
    assert "MICROSERVICE_BAD_DATA" in src and "seldonMessages" in src
    assert "byrow = TRUE" in src  # tensor values are row-major
    for dep in ("plumber", "optparse", "urltools", "stringi"):
        assert f"library({dep})" not in src
    run = _read(os.path.join(ROOT, "wrappers", "R", "s2i", "bin", "run"))
    assert "Rscript /wrapper/microservice.R --model \"$MODEL_NAME\"" in run
    for app in ("MyModel.R", "MyRouter.R", "MyTransformer.R"):
        assert "initialise_seldon <- function(params)" in _read(os.path.join(ROOT, "wrappers", "R", "test", app))


def test_java_wrapper_routes_and_rules():
    src = _read(os.path.join(JAVA_DIR, "Microservice.java"))
    routes = {m.group(1): set(re.findall(r'"(/[a-z-]+)"', m.group(2)))
              for m in re.finditer(r'ROUTES\.put\("(\w+)", Arrays\.asList\(([^)]*)\)\)', src)}
    assert routes == EXPECTED
    for path in {p for ps in EXPECTED.values() for p in ps}:
        assert f'case "{path}":' in src, path
    for t in ('case "INT"', 'case "FLOAT"', 'case "DOUBLE"', 'case "BOOL"'):
        assert t in src, t
    assert 'formField(body, "json")' in src and 'formField(query, "json")' in src
    assert "MICROSERVICE_BAD_DATA" in src and "PREDICTIVE_UNIT_SERVICE_PORT" in src
    # JDK only: no third-party imports anywhere in the wrapper
    for f in os.listdir(JAVA_DIR):
        for imp in re.findall(r"^import ([\w.]+);", _read(os.path.join(JAVA_DIR, f)), re.M):
            assert imp.startswith(("java.", "com.sun.net.httpserver.")) or imp.startswith("io.seldon.amd."), imp
    iface = _read(os.path.join(JAVA_DIR, "SeldonComponent.java"))
    for m in ("predict", "transformInput", "transformOutput", "route", "aggregate", "sendFeedback", "classNames",
              "tags", "metrics"):
        assert re.search(rf"default [\w<>\[\], ]+ {m}\(", iface), m
    run = _read(os.path.join(ROOT, "wrappers", "java", "s2i", "bin", "run"))
    assert "io.seldon.amd.wrapper.Microservice \"$MODEL_NAME\"" in run


def test_java_sources_balance_braces():
    """No javac here: a cheap structural check that every file's braces and
    parentheses balance outside string/char literals."""
    for f in os.listdir(JAVA_DIR) + ["../../../../../../../test/ExampleModel.java"]:
        text = _read(os.path.normpath(os.path.join(JAVA_DIR, f)))
        text = re.sub(r"'(\\.|[^'\\])'", "''", text)  # char literals first: '"' is one
        text = re.sub(r'"(\\.|[^"\\])*"', '""', text)
        text = re.sub(r"//[^\n]*|/\*.*?\*/", "", text, flags=re.S)
        for o, c in ("{}", "()", "[]"):
            assert text.count(o) == text.count(c), (f, o)


@pytest.mark.parametrize("lang,model", [("R", "MyModel.R"), ("java", "ExampleModel")])
def test_builder_contexts(tmp_path, lang, model):
    sys.path.insert(0, ROOT)
    from seldon_core_amd import builder

    src = tmp_path / "src"
    src.mkdir()
    (src / "readme.txt").write_text("x")
    env = {"MODEL_NAME": model, "API_TYPE": "REST", "SERVICE_TYPE": "MODEL", "PERSISTENCE": "0", "LANGUAGE": lang}
    df = builder.write_context(str(src), str(tmp_path / "ctx"), env)
    text = _read(df)
    assert ("Rscript /wrapper/microservice.R" if lang == "R" else "io.seldon.amd.wrapper.Microservice") in text
    assert os.path.isdir(tmp_path / "ctx" / "wrapper") and not os.path.exists(tmp_path / "ctx" / "wrapper" / "test")
    with pytest.raises(builder.BuildError, match="REST only"):
        builder.write_context(str(src), str(tmp_path / "ctx2"), dict(env, API_TYPE="GRPC"))
