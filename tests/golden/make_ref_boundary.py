"""Extract the reference's own boundary test vectors into tests/golden/ref_boundary.json (run in
the build container only; the reference does not exist on the GPU box).

The values are read out of the reference's test files with the `ast` module — literal inputs and
the literal values those tests assert — nothing of the reference is imported or executed:
  backend/tests/test_gemini_rag.py:40-53  citation extraction on an empty / metadata-less /
                                          chunk-less response -> []
  backend/tests/test_gemini_rag.py:55-72  the grounding chunk a response carries and the
                                          citation dict the adapter must build from it
  backend/tests/test_gemini_rag.py:85-93  stream ids: two distinct 36-character strings
  backend/tests/test_chat_stream_helpers.py:37-59  citation -> "source-document" SSE payload
  backend/tests/test_chat_stream_helpers.py:62-75  "finish" SSE payload

Usage: python tests/golden/make_ref_boundary.py [/root/reference]
"""
import ast
import json
import os
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def fn(tree, name):
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == name:
            return node
    raise KeyError(name)


def kwargs(call):
    return {k.arg: k.value for k in call.keywords}


def calls(node, func_name):
    return [n for n in ast.walk(node) if isinstance(n, ast.Call) and getattr(n.func, "id", None) == func_name]


def path_of(sub):
    """citations[0]["uri"] -> ["citations", 0, "uri"]"""
    out = []
    while isinstance(sub, ast.Subscript):
        out.append(ast.literal_eval(sub.slice))
        sub = sub.value
    out.append(sub.id)
    return out[::-1]


def asserted_equalities(node):
    """assert <subscript chain> == <literal> / assert len(x) == <literal>, in source order."""
    out = []
    for a in (n for n in ast.walk(node) if isinstance(n, ast.Assert)):
        t = a.test
        if not (isinstance(t, ast.Compare) and len(t.ops) == 1 and isinstance(t.ops[0], ast.Eq)):
            continue
        lhs, rhs = t.left, t.comparators[0]
        try:
            val = ast.literal_eval(rhs)
        except ValueError:
            continue
        if isinstance(lhs, ast.Subscript):
            out.append({"path": path_of(lhs), "equals": val, "line": a.lineno})
        elif isinstance(lhs, ast.Call) and getattr(lhs.func, "id", None) == "len":
            out.append({"len_of": lhs.args[0].id, "equals": val, "line": a.lineno})
    return sorted(out, key=lambda e: e["line"])


def main():
    p1 = os.path.join(REF, "backend/tests/test_gemini_rag.py")
    p2 = os.path.join(REF, "backend/tests/test_chat_stream_helpers.py")
    t1 = ast.parse(open(p1).read())
    t2 = ast.parse(open(p2).read())

    valid = fn(t1, "test_extract_citations_returns_valid_structure")
    rc_call = [c for c in calls(valid, "Mock") if "retrieved_context" in kwargs(c)][0]
    chunk = {"retrieved_context": {k: ast.literal_eval(v) for k, v in kwargs(kwargs(rc_call)["retrieved_context"]).items()},
             "web": ast.literal_eval(kwargs(rc_call)["web"])}

    ids = fn(t1, "test_new_stream_ids_returns_unique_ids")
    id_len = sorted({c["equals"] for c in asserted_equalities(ids) if "len_of" in c})

    frames = fn(t2, "test_citation_frames_preserve_source_document_wire_format")
    lam = [n for n in ast.walk(frames) if isinstance(n, ast.Lambda)][0]
    citation_in = ast.literal_eval(lam.body)[0]
    payload_cmp = [a.test for a in ast.walk(frames) if isinstance(a, ast.Assert) and isinstance(a.test, ast.Compare)
                   and isinstance(a.test.comparators[0], ast.Dict)][0]
    frame_out = ast.literal_eval(payload_cmp.comparators[0])

    fin = fn(t2, "test_finish_frame_exposes_frontend_usage_contract")
    fin_call = [n for n in ast.walk(fin) if isinstance(n, ast.Call) and getattr(n.func, "attr", None) == "_finish_frame"][0]
    fin_in = {k: ast.literal_eval(v) for k, v in kwargs(fin_call).items()}
    fin_eq = asserted_equalities(fin)

    empty_cases = [n for n in ("test_extract_citations_handles_empty_response",
                               "test_extract_citations_handles_missing_metadata",
                               "test_extract_citations_handles_missing_chunks")]
    for n in empty_cases:
        fn(t1, n)  # present in the reference

    out = {
        "source": "ast literals of the reference's boundary tests (tests/golden/make_ref_boundary.py)",
        "extract_citations_valid": {
            "source": f"backend/tests/test_gemini_rag.py:{valid.lineno}-{valid.end_lineno}",
            "grounding_chunk": chunk,
            "asserts": asserted_equalities(valid),
        },
        "extract_citations_empty": {
            "source": "backend/tests/test_gemini_rag.py:40-53",
            "cases": ["candidates=[]", "grounding_metadata=None", "grounding_chunks=None"],
            "expect": [],
        },
        "stream_ids": {"source": f"backend/tests/test_gemini_rag.py:{ids.lineno}-{ids.end_lineno}", "length": id_len},
        "citation_frame": {
            "source": f"backend/tests/test_chat_stream_helpers.py:{frames.lineno}-{frames.end_lineno}",
            "citation": citation_in, "payload": frame_out,
        },
        "finish_frame": {
            "source": f"backend/tests/test_chat_stream_helpers.py:{fin.lineno}-{fin.end_lineno}",
            "kwargs": fin_in, "asserts": fin_eq,
        },
    }
    with open(os.path.join(HERE, "ref_boundary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1)[:1500])


if __name__ == "__main__":
    main()
