"""CPU oracle for the rfx retrieval path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / CPU baseline.  The product path
(``rag-foundation_amd/rfx``) never imports it and fails loudly when the HIP library is missing.

What it restates (reference = Sapphire-Bridge/rag-foundation, paths relative to its root):
  * textproc.normalize          scripts/benchmark/metrics.py:13-19 (``_normalize``)
  * textproc.contents_to_text   backend/app/services/gemini_rag.py:640-654
  * mock_ref.*                  backend/app/services/gemini_rag.py:554-595, 602-718;
                                backend/app/routes/chat.py:576-603 (SSE citation / finish payloads)
  * search.topk_blocks          search.topk over corpora streamed block by block (full-size checks)
  * chunk/featurize/embed/search: the reference performs these remotely (Gemini File Search,
    gemini_rag.py:319-327, 463-469, 536); there is no reference arithmetic to follow, so these
    are the build's own definitions — "parity unpinned" against Gemini.

Pinning:
  * the tokenizer: tests/golden/ref_normalize.json, outputs of the reference's own
    scripts/benchmark/metrics.py (imported directly, standard library only;
    tests/golden/make_ref_golden.py);
  * citation extraction and the SSE payloads: tests/golden/ref_boundary.json, the inputs and
    asserted values of the reference's tests (backend/tests/test_gemini_rag.py:40-93,
    backend/tests/test_chat_stream_helpers.py:37-75), extracted with `ast` by
    tests/golden/make_ref_boundary.py;
  * the mock's response shape (mock_response, first_stream_text, contents -> question): the
    reference MockGeminiRag's own outputs for a fixed question list, tests/golden/ref_mock.json
    (captured by importing it in the build container, tests/golden/make_ref_mock.py);
  * the exact two-pass scan (screen.py): its int8 copy bit-exact on the GPU, its selection rule shown
    on the CPU to return search.topk exactly (tests/test_screen_oracle.py);
  * the numeric path (synth/embed/search): no reference counterpart — parity unpinned against
    Gemini; pinned by its own committed fixtures (tests/golden/make_golden.py) and exact-arithmetic
    identities.
"""
