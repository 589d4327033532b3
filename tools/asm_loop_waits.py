"""Dev tool: count the vmcnt waits hipcc itself inserted (outside inline asm) from each kernel's
first loop header on, in a hipcc -save-temps gfx950 .s file.  A kernel that streams by asm
LDS-DMA must show 0: a compiler wait counts the DMA ops too and drains the ring (k_mfma_common.h
launder)."""
import re
import sys

for path in sys.argv[1:]:
    s = open(path).read()
    for m in re.finditer(r"^(_ZN3rfx\S+):[^\n]*\n(.*?)^\.Lfunc_end", s, re.S | re.M):
        name, body = m.group(1), m.group(2)
        lines = body.split("\n")
        hdr = [i for i, line in enumerate(lines) if "Loop Header" in line]
        if not hdr:
            continue
        inasm, cnt = False, 0
        for line in lines[hdr[0]:]:
            if "ASMSTART" in line:
                inasm = True
            elif "ASMEND" in line:
                inasm = False
            elif "s_waitcnt" in line and "vmcnt" in line and not inasm:
                cnt += 1
        print(f"{cnt:4d}  {name[:90]}")
