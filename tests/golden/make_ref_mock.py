"""Generate tests/golden/ref_mock.json: outputs of the reference's own mock retriever
(MockGeminiRag, backend/app/services/gemini_rag.py:602-718), captured by importing it in the BUILD
container.  The reference's code never ships: only this JSON (data) is committed.

The import needs two third-party modules this image lacks: `tenacity` (the retry
decorator gemini_rag.py:10 applies to the real client) and `pydantic_settings` (app/config.py).
Throwaway stand-ins are written to a temporary directory that is deleted afterwards; neither is on
the mock's code path (no retry fires in the mock, and the settings only select the mock).

UUIDs in names are reduced to their pattern ("<hex32>") so the fixture is deterministic.
Run: python tests/golden/make_ref_mock.py  (build container; /root/reference must exist)
"""
import json
import os
import re
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF_BACKEND = "/root/reference/backend"
SAMPLE = "/root/reference/docs/demo/sample-report.md"

TENACITY = '''
def retry(*a, **k):
    def deco(f):
        return f
    return deco
def stop_after_attempt(*a, **k): return None
def wait_exponential(*a, **k): return None
def retry_if_exception(*a, **k): return None
def retry_if_exception_type(*a, **k): return None
'''
PYDANTIC_SETTINGS = '''
from pydantic import BaseModel, ConfigDict
BaseSettings = BaseModel
def SettingsConfigDict(**kw):
    return ConfigDict(extra="ignore")
'''

HEX32 = re.compile(r"[0-9a-f]{32}")


def scrub(s):
    return HEX32.sub("<hex32>", s) if isinstance(s, str) else s


def ns_to_dict(o, depth=0):
    """SimpleNamespace / list / scalar -> JSON-able structure (attribute names kept)."""
    if depth > 12:
        return repr(o)
    if isinstance(o, (str, int, float, bool)) or o is None:
        return scrub(o)
    if isinstance(o, (list, tuple)):
        return [ns_to_dict(x, depth + 1) for x in o]
    if isinstance(o, dict):
        return {k: ns_to_dict(v, depth + 1) for k, v in o.items()}
    if hasattr(o, "__dict__"):
        return {"__type__": type(o).__name__, **{k: ns_to_dict(v, depth + 1) for k, v in vars(o).items()}}
    return repr(o)


def main():
    questions = json.load(open(os.path.join(HERE, "bench_questions.json")))["questions"]
    extra = ["", "   ", "x" * 200, "Ünïcödé question — with dashes?"]
    with tempfile.TemporaryDirectory() as shim:
        with open(os.path.join(shim, "tenacity.py"), "w") as f:
            f.write(TENACITY)
        os.makedirs(os.path.join(shim, "pydantic_settings"))
        with open(os.path.join(shim, "pydantic_settings", "__init__.py"), "w") as f:
            f.write(PYDANTIC_SETTINGS)
        sys.path[:0] = [shim, REF_BACKEND]
        sys.dont_write_bytecode = True
        from app.services import gemini_rag as g  # noqa: E402  (reference, imported as data source)

        client = g.get_rag_client()
        out = {"source": "backend/app/services/gemini_rag.py:602-725 (MockGeminiRag), captured by "
                         "tests/golden/make_ref_mock.py",
               "client_type": type(client).__name__, "is_mock": bool(getattr(client, "is_mock", False))}
        store = client.create_store("demo")
        up = client.upload_file(store, SAMPLE, display_name="sample-report.md")
        out["create_store"] = scrub(store)
        out["upload_file"] = {"operation_name": scrub(up.operation_name), "file_id": scrub(up.file_id)}
        out["op_status"] = ns_to_dict(client.op_status(up.operation_name))
        out["op_status"]["name"] = scrub(out["op_status"]["name"])
        out["op_status_dict_input"] = ns_to_dict(client.op_status({"name": up.operation_name}))
        cases = []
        for q in questions + extra:
            for stores in ([store], [], [store, "fileSearchStores/other"]):
                contents = [{"role": "user", "parts": [{"text": "earlier turn"}]},
                            {"role": "model", "parts": [{"text": "answer"}]},
                            {"role": "user", "parts": [{"text": q}]}]
                chunks = list(client.ask_stream(contents=contents, store_names=stores, metadata_filter=None,
                                                model="gemini-2.5-flash"))
                resp = client.ask(contents=contents, store_names=stores, metadata_filter=None,
                                  model="gemini-2.5-flash")
                cases.append({
                    "question": q, "store_names": [scrub(s) for s in stores],
                    "contents_to_text": client._contents_to_text(contents),
                    "stream": [ns_to_dict(c) for c in chunks],
                    "ask": ns_to_dict(resp),
                    "citations": [{k: scrub(v) for k, v in c.items()}
                                  for c in g.GeminiRag.extract_citations_from_response(chunks[-1])],
                })
        out["cases"] = cases
        # contents shapes the chat route never sends but the extractor accepts
        out["contents_to_text_shapes"] = [
            {"contents": c, "text": client._contents_to_text(c)}
            for c in ["plain string", ["a", "  ", "last"], [{"parts": [{"text": "  spaced  "}]}], [], 42]]
        ids = g.GeminiRag.new_stream_ids() if hasattr(g.GeminiRag, "new_stream_ids") else None
        out["new_stream_ids_pattern"] = [HEX32.sub("<hex32>", x.replace("-", "")) for x in ids] if ids else None
    path = os.path.join(HERE, "ref_mock.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, ensure_ascii=False)
    print(f"wrote {path}: {len(out['cases'])} cases")


if __name__ == "__main__":
    main()
