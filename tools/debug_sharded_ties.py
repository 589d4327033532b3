"""Dev tool: the screened store of tests/test_gpu_sharded.py (repetitive documents: many exactly tied
rows) searched plain, sharded (0x4) and per shard, each against a numpy f64 restatement of the
ranking rule (score desc, row asc; scores are the f32 rounding of the exact dot).  Prints every
mismatch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rag-foundation_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["RFX_SCREEN"] = "1"
import tempfile  # noqa: E402

import torch  # noqa: E402

from rfx import filters  # noqa: E402
from rfx import store as rstore  # noqa: E402
from rfx.retriever import GpuRetriever  # noqa: E402

DOCS = [("alpha beta gamma delta epsilon " * 40, {"tenant": "acme"}),
        ("zeta eta theta iota kappa lambda " * 35, {"tenant": "globex"}),
        ("mock mode document assistant retrieval citations " * 30, {"tenant": "acme"}),
        ("hbm bandwidth roofline matrix cores wavefront lds " * 33, None)]
QUESTIONS = ["alpha gamma", "theta kappa lambda", "document retrieval", "roofline lds", "beta zeta assistant"]

root = tempfile.mkdtemp()
writer = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0), dtype="bf16")
name = writer.create_store("shared")
for i, (t, m) in enumerate(DOCS):
    writer.add_document(name, t, f"doc{i}", {"white_space_config": {"max_tokens_per_chunk": 4}}, m)
plain = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0), dtype="bf16")
pst = plain.registry.get(name)
sharded = GpuRetriever(registry=rstore.StoreRegistry(root=root, device=0, devices="0x4"), dtype="bf16")
sst = sharded.registry.get(name)
six = sst.index
X = pst.index.read(0, pst.index.rows).float().cpu().numpy().astype(np.float64)
print("rows", X.shape[0], "bases", six.bases, "shard rows", [s.rows for s in six.shards])
emb = plain.embedder(768)
bad = 0
for qq in QUESTIONS:
    q = emb.embed_texts([qq], "bf16")
    q64 = q.float().cpu().numpy().astype(np.float64)[0]
    for filt in (None, {"tenant": "acme"}):
        k = 7
        if filt is None:
            allowed = np.ones(X.shape[0], bool)
            pm = sm = None
        else:
            ranges = pst.mask_ranges(filt)
            allowed = np.zeros(X.shape[0], bool)
            for a, n in ranges:
                allowed[a:a + n] = True
            words = filters.row_mask_words(pst.index.rows, ranges)
            pm = torch.from_numpy(words).cuda()
            sm = six.mask_tensor(words)
        sc = (X @ q64).astype(np.float32)
        idx = np.nonzero(allowed)[0]
        order = idx[np.lexsort((idx, -sc[idx].astype(np.float64)))][:k]
        ps, pr = pst.index.search(q, k, row_mask=pm)
        ss, sr = six.search(q, k, row_mask=sm)
        pr, sr = pr.cpu().numpy()[0], sr.cpu().numpy()[0]
        tag = f"{qq!r} filt={filt}"
        if not np.array_equal(pr, order):
            bad += 1
            print("PLAIN  ", tag, "got", pr.tolist(), "want", order.tolist(), "scores", sc[order].tolist())
        if not np.array_equal(sr, order):
            bad += 1
            print("SHARDED", tag, "got", sr.tolist(), "want", order.tolist())
            for i, (sh, base) in enumerate(zip(six.shards, six.bases)):
                lo, hi = base, base + sh.rows
                li = idx[(idx >= lo) & (idx < hi)]
                want = li[np.lexsort((li, -sc[li].astype(np.float64)))][:k]
                rec = sh.search_records(q, k, row_offset=base, row_mask=sm[i] if sm is not None else None)
                got = rec[0, :, 1].cpu().numpy()
                print(f"   shard {i} [{lo},{hi}) plan {sh.search_plan(1, k)} got {got.tolist()} want {want.tolist()}")
print("mismatches", bad)
