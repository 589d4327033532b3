"""Generate golden vectors FROM THE REFERENCE (run in the build container only; the reference
does not exist on the GPU box).  Output files are committed data fixtures:

  ref_normalize.json   inputs -> reference scripts/benchmark/metrics.py:_normalize outputs
                       (the module imports only the standard library, so it is imported directly
                       from /root/reference; nothing is stubbed)
  sample_report.md     docs/demo/sample-report.md (BASELINE config 1 input document, data)
  bench_questions.json scripts/benchmark/datasets/sample/questions.jsonl questions (data)
  ref_citation_hit.json inputs -> reference scripts/benchmark/metrics.py:citation_hit outputs
                       (citation dicts shaped as run_benchmark.py:209-216 parses them)

Usage: python tests/golden/make_ref_golden.py [/root/reference]
"""
import importlib.util
import json
import os
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [
    "", "Hello, World!", "The quick brown fox jumps over a lazy dog.", "an apple a day",
    "RAG Foundation is a mock-mode document assistant", "UPPER lower MiXeD 123 4x5",
    "tabs\tand\nnewlines\r\nand  double  spaces", "punct:;,.!?()[]{}<>\"'`~@#$%^&*-_=+|\\/",
    "numbers 3.14159 and 2,718 and -42", "unicode café naïve résumé Ünïcödé",
    "emoji 🚀 rocket and ✓ check", "İstanbul KELVIN K sign", "ＦＵＬＬＷＩＤＴＨ ａｂｃ",
    "the the the", "a", "A An THE", "non breaking space", "snake_case and kebab-case",
    "e-mail: someone@example.com, url https://example.com/a?b=c",
    "What is the purpose of the /api/chat endpoint in this service?",
    "Who wrote the song \"CompletelyMadeUpTitleXYZ\"?",
]


def main():
    spec = importlib.util.spec_from_file_location("ref_metrics", os.path.join(REF, "scripts/benchmark/metrics.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sample = open(os.path.join(REF, "docs/demo/sample-report.md"), encoding="utf-8").read()
    qs = [json.loads(l)["question"] for l in open(os.path.join(REF, "scripts/benchmark/datasets/sample/questions.jsonl"))
          if l.strip()]
    cases = CASES + sample.splitlines() + [sample] + qs
    out = [{"input": c, "normalized": mod._normalize(c)} for c in cases]
    with open(os.path.join(HERE, "ref_normalize.json"), "w") as f:
        json.dump({"source": "scripts/benchmark/metrics.py:13-19 (_normalize), imported from the reference",
                   "cases": out}, f, indent=1, ensure_ascii=False)
    with open(os.path.join(HERE, "sample_report.md"), "w", encoding="utf-8") as f:
        f.write(sample)
    with open(os.path.join(HERE, "bench_questions.json"), "w") as f:
        json.dump({"source": "scripts/benchmark/datasets/sample/questions.jsonl", "questions": qs}, f, indent=1)
    hit_cases = [
        ([], ["a.md"]), ([{"title": "a.md"}], []), ([{"title": "A.MD"}], ["a.md"]),
        ([{"title": "b.md", "sourceId": "cit-0"}], ["b.md"]), ([{"title": "b.md", "sourceId": "cit-0"}], ["cit-0"]),
        ([{"sourceId": "cit-1", "title": "x"}, {"title": "y"}], ["y"]), ([{"uri": "local://s/f#chunk-3"}], ["local://s/f#chunk-3"]),
        ([{"doc_id": "D1", "title": "t"}], ["d1"]), ([{"title": None, "snippet": "s"}], ["s"]),
        ([{"title": "sample-report.md", "snippet": "x", "sourceId": "cit-0"}, {"title": "other.md", "sourceId": "cit-1"}],
         ["sample-report.md", "other.md"]),
    ]
    hits = [{"citations": c, "gold": g, "citation_hit": mod.citation_hit(c, g)} for c, g in hit_cases]
    with open(os.path.join(HERE, "ref_citation_hit.json"), "w") as f:
        json.dump({"source": "scripts/benchmark/metrics.py:73-92 (citation_hit), imported from the reference",
                   "cases": hits}, f, indent=1)
    print(f"wrote {len(out)} normalize cases, sample report ({len(sample)} B), {len(qs)} questions, "
          f"{len(hits)} citation_hit cases")


if __name__ == "__main__":
    main()
