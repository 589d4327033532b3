"""Per-kernel statistics from a hipcc -save-temps gfx950 .s file (dev tool, not product)."""
import re
import sys


def kernels(text):
    out = {}
    for m in re.finditer(r"^(\S+):\s*; @\1\n(.*?)^\s*s_endpgm", text, re.S | re.M):
        out[m.group(1)] = m.group(2)
    return out


def meta(text):
    res = {}
    for blk in re.findall(r"(- \.agpr_count:.*?\.wavefront_size:\s+\d+)", text, re.S):
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        d = {}
        for key in ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size",
                    "private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count"):
            mm = re.search(r"\." + key + r":\s+(\d+)", blk)
            if mm:
                d[key] = int(mm.group(1))
        res[name] = d
    return res


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    md = meta(text)
    for name, body in kernels(text).items():
        if pat not in name:
            continue
        cnt = {p: len(re.findall(p, body)) for p in
               ("global_load_lds", "v_mfma", "s_barrier", "ds_read", "ds_write", "scratch_",
                "buffer_load", "global_load_dword", "s_waitcnt vmcnt")}
        waits = sorted(set(re.findall(r"s_waitcnt vmcnt\(\d+\)", body)))
        print(name[:90])
        print("   ", md.get(name, {}), "lines", body.count("\n"))
        print("   ", cnt, waits)
