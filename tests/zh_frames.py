"""Header-level walker of RFC 8878 frames (test infrastructure): lists, per block, the
block type, literals-section type / stream count / Huffman weight encoding and the
three sequence-table modes, so the tests can show which decoder paths a set of frames
exercises.  Nothing is decoded."""

LIT_TYPES = ("raw", "rle", "huffman", "treeless")
SEQ_MODES = ("predefined", "rle", "fse", "repeat")


def walk(frame: bytes):
    """-> list of per-block dicts; raises ValueError on a malformed header."""
    b = frame
    ip, blocks = 0, []
    while ip < len(b):
        magic = int.from_bytes(b[ip:ip + 4], "little")
        if magic & 0xFFFFFFF0 == 0x184D2A50:
            ip += 8 + int.from_bytes(b[ip + 4:ip + 8], "little")
            blocks.append({"type": "skippable"})
            continue
        if magic != 0xFD2FB528:
            raise ValueError("bad magic")
        fhd = b[ip + 4]
        single, chk, did, fcsf = (fhd >> 5) & 1, (fhd >> 2) & 1, fhd & 3, fhd >> 6
        hs = 1 + (0 if single else 1) + (0, 1, 2, 4)[did] + ((1 if single else 0), 2, 4, 8)[fcsf]
        dp = ip + 5 + (0 if single else 1)
        dict_id = int.from_bytes(b[dp:dp + (0, 1, 2, 4)[did]], "little")
        ip += 4 + hs
        first = True
        while True:
            bh = int.from_bytes(b[ip:ip + 3], "little")
            last, bt, bsz = bh & 1, (bh >> 1) & 3, bh >> 3
            ip += 3
            d = {"type": ("raw", "rle", "compressed", "reserved")[bt], "size": bsz, "first_in_frame": first, "checksum": bool(chk),
                 "single_segment": bool(single), "fcs": fcsf != 0 or bool(single), "dict_id": dict_id}
            first = False
            if bt == 2:
                p = b[ip:ip + bsz]
                lt, sf = p[0] & 3, (p[0] >> 2) & 3
                d["lit"] = LIT_TYPES[lt]
                if lt <= 1:
                    lhs = 1 if sf in (0, 2) else sf
                    n = p[0] >> 3 if lhs == 1 else (int.from_bytes(p[:lhs], "little") >> 4)
                    sec = lhs + (n if lt == 0 else 1)
                else:
                    lhs = 3 if sf <= 1 else sf + 2
                    h = int.from_bytes(p[:lhs], "little")
                    nb = 10 if sf <= 1 else 14 if sf == 2 else 18
                    cs = (h >> (4 + nb)) & ((1 << nb) - 1)
                    d["streams"] = 1 if sf == 0 else 4
                    if lt == 2:
                        d["weights"] = "fse" if p[lhs] < 128 else "direct"
                    sec = lhs + cs
                s = p[sec:]
                nseq = s[0]
                if nseq == 0:
                    d["nseq"] = 0
                else:
                    k = 1 if nseq < 128 else 2 if nseq < 255 else 3
                    d["nseq"] = nseq if k == 1 else (((nseq - 128) << 8) + s[1] if k == 2 else s[1] + (s[2] << 8) + 0x7F00)
                    m = s[k]
                    d["modes"] = (SEQ_MODES[m >> 6], SEQ_MODES[(m >> 4) & 3], SEQ_MODES[(m >> 2) & 3])
                ip += bsz
            elif bt == 1:
                ip += 1
            else:
                ip += bsz
            blocks.append(d)
            if last:
                break
        if chk:
            ip += 4
    return blocks


def features(frames):
    """Set of decoder paths the frames exercise."""
    f = set()
    for fr in frames:
        for d in walk(fr):
            f.add("block_" + d["type"])
            if d.get("checksum"):
                f.add("checksum")
            if not d.get("fcs", True):
                f.add("no_fcs")
            if "single_segment" in d and not d["single_segment"]:
                f.add("window_descriptor")
            if d["type"] == "compressed":
                f.add("lit_" + d["lit"])
                if "streams" in d:
                    f.add(f"huf_{d['streams']}stream")
                if "weights" in d:
                    f.add("weights_" + d["weights"])
                if d.get("nseq", 0) == 0:
                    f.add("no_sequences")
                for t, m in zip(("ll", "of", "ml"), d.get("modes", ())):
                    f.add(f"{t}_{m}")
    return f
