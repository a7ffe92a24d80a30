"""The Go binding (go/split/gpusplit.go) is not built here (no Go toolchain), so these CPU
checks keep it self-consistent: INTEGRATION.md quotes the committed file verbatim, every method
it calls on the GPUWriter is defined, every C entry point it calls is declared in
include/bsgpu.h, and each chunk reaches the store through exactly one Put, inside F
(the earlier stub called undefined helpers and Put chunks twice)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "split", "gpusplit.go")


def _src() -> str:
    with open(GO) as f:
        return f.read()


def test_integration_quotes_the_file():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        doc = f.read()
    assert "```go\n" + _src() + "```\n" in doc


def test_methods_and_c_calls_defined():
    src = _src()
    defined = set(re.findall(r"func \(w \*GPUWriter\) (\w+)\(", src))
    called = set(re.findall(r"\bw\.(\w+)\(", src))
    # fields holding interfaces / objects whose methods are called
    called -= {"rp", "st", "tb"}
    assert called <= defined, called - defined
    with open(os.path.join(ROOT, "include", "bsgpu.h")) as f:
        header = f.read()
    for fn in set(re.findall(r"\bC\.(bsg_\w+)\(", src)):
        assert re.search(r"\b%s\(" % fn, header), fn
    for const in set(re.findall(r"\bC\.(BSG_\w+)\b", src)):
        assert "#define " + const in header, const


def test_each_chunk_put_once_inside_f():
    src = _src()
    f_body = src[src.index("func (w *GPUWriter) newTreeBuilder()"):src.index("// Write implements")]
    assert "w.rp.PutWithRef(" in f_body and "w.st.Put(" in f_body
    # outside F nothing Puts a chunk: drain only records the ref and calls tb.Add
    rest = src.replace(f_body, "")
    assert "PutWithRef(w.Ctx" not in rest and "st.Put(" not in rest
    drain = src[src.index("func (w *GPUWriter) drain()"):src.index("// Close implements")]
    assert "w.tb.Add(" in drain and "w.refs[&chunk[0]] =" in drain
