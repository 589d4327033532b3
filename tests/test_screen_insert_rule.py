"""CPU: the list-insert rule of kernel 10's slow path (k_scan_screen.h fold_screen), restated.

The kernel inserts a key into a lane's sorted list L (descending, 64-bit keys, 0 = empty) without a
dependency chain: with c_i = (L_i > key), the new entry i is c_{i-1} ? (c_i ? L_i : key) : L_{i-1}
(c_{-1} = true), and what falls out is c_{KL-1} ? key : L_{KL-1}.  That must equal the top KL of
L + [key] and the smallest of them, for keys that tie with entries too (ties cannot occur in the
kernel — the row is in the key's low bits — but the rule does not need that)."""
import random

import pytest


def chain_free_insert(L, key):
    kl = len(L)
    c = [L[i] > key for i in range(kl)]
    fallen = key if c[kl - 1] else L[kl - 1]
    new = [0] * kl
    for i in range(kl - 1, 0, -1):
        new[i] = (L[i] if c[i] else key) if c[i - 1] else L[i - 1]
    new[0] = L[0] if c[0] else key
    return new, fallen


@pytest.mark.parametrize("kl", [4, 10])
def test_insert_rule_matches_sorted_top_kl(kl):
    rng = random.Random(kl)
    for _ in range(3000):
        fill = rng.randint(0, kl)
        L = sorted((rng.randint(1, 50) for _ in range(fill)), reverse=True) + [0] * (kl - fill)
        key = rng.randint(1, 50)
        new, fallen = chain_free_insert(L, key)
        every = sorted(L + [key], reverse=True)
        assert new == every[:kl] and fallen == every[kl]
