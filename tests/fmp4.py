"""Test helper: rewrite a progressive MP4 (moov sample tables) as a fragmented
MP4 (ISO/IEC 14496-12 §8.8: moov with empty sample tables + mvex/trex, then
moof/mdat pairs) holding the same samples, so the demuxer's fragment path can
be checked against the progressive file it came from.  Plain Python, test
infrastructure only."""
from __future__ import annotations

import struct
from pathlib import Path


def _boxes(b: bytes, off: int, end: int):
    while off + 8 <= end:
        size, typ = struct.unpack(">I4s", b[off:off + 8])
        hdr = 8
        if size == 1:
            size = struct.unpack(">Q", b[off + 8:off + 16])[0]
            hdr = 16
        elif size == 0:
            size = end - off
        yield typ.decode("latin1"), off, off + hdr, off + size
        off += size


def _child(b, s, e, typ, skip=0):
    for t, o, ps, pe in _boxes(b, s + skip, e):
        if t == typ:
            return o, ps, pe
    return None


def _box(typ: str, payload: bytes) -> bytes:
    return struct.pack(">I4s", 8 + len(payload), typ.encode()) + payload


def _full(typ: str, ver: int, flags: int, payload: bytes) -> bytes:
    return _box(typ, struct.pack(">I", (ver << 24) | flags) + payload)


def _samples(b: bytes, stbl: tuple) -> dict:
    _, s, e = stbl
    r = {}
    _, ps, pe = _child(b, s, e, "stsz")
    uni, n = struct.unpack(">II", b[ps + 4:ps + 12])
    sizes = [uni] * n if uni else list(struct.unpack(">%dI" % n, b[ps + 12:ps + 12 + 4 * n]))
    c = _child(b, s, e, "stco")
    if c:
        nc = struct.unpack(">I", b[c[1] + 4:c[1] + 8])[0]
        chunks = list(struct.unpack(">%dI" % nc, b[c[1] + 8:c[1] + 8 + 4 * nc]))
    else:
        c = _child(b, s, e, "co64")
        nc = struct.unpack(">I", b[c[1] + 4:c[1] + 8])[0]
        chunks = list(struct.unpack(">%dQ" % nc, b[c[1] + 8:c[1] + 8 + 8 * nc]))
    _, ps, _ = _child(b, s, e, "stsc")
    ne = struct.unpack(">I", b[ps + 4:ps + 8])[0]
    ents = [struct.unpack(">III", b[ps + 8 + 12 * i:ps + 20 + 12 * i]) for i in range(ne)]
    offs, k = [], 0
    for i, (first, spc, _) in enumerate(ents):
        last = ents[i + 1][0] if i + 1 < ne else len(chunks) + 1
        for ch in range(first, last):
            o = chunks[ch - 1]
            for _ in range(spc):
                if k >= n:
                    break
                offs.append(o)
                o += sizes[k]
                k += 1
    _, ps, _ = _child(b, s, e, "stts")
    ne = struct.unpack(">I", b[ps + 4:ps + 8])[0]
    durs = []
    for i in range(ne):
        cnt, d = struct.unpack(">II", b[ps + 8 + 8 * i:ps + 16 + 8 * i])
        durs += [d] * cnt
    cto = [0] * n
    c = _child(b, s, e, "ctts")
    if c:
        ne = struct.unpack(">I", b[c[1] + 4:c[1] + 8])[0]
        k = 0
        for i in range(ne):
            cnt, o = struct.unpack(">Ii", b[c[1] + 8 + 8 * i:c[1] + 16 + 8 * i])
            for _ in range(cnt):
                cto[k] = o
                k += 1
    sync = [1] * n
    c = _child(b, s, e, "stss")
    if c:
        ne = struct.unpack(">I", b[c[1] + 4:c[1] + 8])[0]
        sync = [0] * n
        for i in struct.unpack(">%dI" % ne, b[c[1] + 8:c[1] + 8 + 4 * ne]):
            sync[i - 1] = 1
    r.update(sizes=sizes, offsets=offs, durations=durs[:n] + [durs[-1] if durs else 0] * (n - len(durs)),
             cto=cto, sync=sync)
    return r


def fragment(src: str | Path, dst: str | Path, *, per_fragment: int = 30, zero_mvhd: bool = False,
             mehd: bool = True, trex_defaults: bool = True) -> dict:
    """Write `dst` as a fragmented copy of progressive `src`: every track's
    samples in runs of `per_fragment` per moof (one traf per track per moof,
    tfhd default-base-is-moof, tfdt, one trun with data_offset and per-sample
    size / flags / composition offsets; durations per sample or, with
    trex_defaults and a constant duration, from trex).  zero_mvhd: mvhd
    duration 0 (the fragments time the file).  Returns the tracks' tables."""
    b = Path(src).read_bytes()
    moov = _child(b, 0, len(b), "moov")
    ftyp = _child(b, 0, len(b), "ftyp")
    tracks = []
    new_moov = b""
    for t, o, ps, pe in _boxes(b, moov[1], moov[2]):
        if t == "mvhd":
            box = bytearray(b[o:pe])
            if zero_mvhd:
                ver = box[8]
                at = 8 + (28 if ver == 1 else 20)
                box[at:at + (8 if ver == 1 else 4)] = b"\0" * (8 if ver == 1 else 4)
            new_moov += bytes(box)
        elif t == "trak":
            tk = _child(b, ps, pe, "tkhd")
            ver = b[tk[1]]
            tid = struct.unpack(">I", b[tk[1] + (12 if ver == 0 else 20):tk[1] + (16 if ver == 0 else 24)])[0]
            mdia = _child(b, ps, pe, "mdia")
            minf = _child(b, mdia[1], mdia[2], "minf")
            stbl = _child(b, minf[1], minf[2], "stbl")
            tab = _samples(b, stbl)
            tab["id"] = tid
            tracks.append(tab)
            stsd = _child(b, stbl[1], stbl[2], "stsd")
            empty = (b[stsd[0]:stsd[2]] + _full("stts", 0, 0, struct.pack(">I", 0)) +
                     _full("stsc", 0, 0, struct.pack(">I", 0)) + _full("stsz", 0, 0, struct.pack(">II", 0, 0)) +
                     _full("stco", 0, 0, struct.pack(">I", 0)))
            new_stbl = _box("stbl", empty)
            # rebuild trak with the emptied stbl (sizes of minf / mdia / trak follow)
            minf_new = b"".join(b[o2:pe2] if t2 != "stbl" else new_stbl for t2, o2, _, pe2 in _boxes(b, minf[1], minf[2]))
            mdia_new = b"".join(b[o2:pe2] if t2 != "minf" else _box("minf", minf_new)
                                for t2, o2, _, pe2 in _boxes(b, mdia[1], mdia[2]))
            trak_new = b"".join(b[o2:pe2] if t2 != "mdia" else _box("mdia", mdia_new)
                                for t2, o2, _, pe2 in _boxes(b, ps, pe))
            new_moov += _box("trak", trak_new)
        else:
            new_moov += b[o:pe]
    mvex = b""
    if mehd:
        mvhd = _child(b, moov[1], moov[2], "mvhd")
        ver = b[mvhd[1]]
        dur = struct.unpack(">Q" if ver == 1 else ">I", b[mvhd[1] + (28 if ver == 1 else 20):
                                                          mvhd[1] + (36 if ver == 1 else 24)])[0]
        mvex += _full("mehd", 1, 0, struct.pack(">Q", dur))
    for tab in tracks:
        d = tab["durations"]
        const = len(set(d)) == 1 and trex_defaults
        tab["const"] = const
        mvex += _full("trex", 0, 0, struct.pack(">IIIII", tab["id"], 1, d[0] if const else 0, 0, 0))
    out = bytearray(b[ftyp[0]:ftyp[2]] + _box("moov", new_moov + _box("mvex", mvex)))
    n_max = max(len(t["sizes"]) for t in tracks)
    seq = 1
    dts = [0] * len(tracks)
    for f0 in range(0, n_max, per_fragment):
        trafs, payload, placements = [], bytearray(), []
        for k, tab in enumerate(tracks):
            idx = list(range(f0, min(f0 + per_fragment, len(tab["sizes"]))))
            if not idx:
                continue
            flags = 0x1 | 0x200 | 0x400 | 0x800 | (0 if tab["const"] else 0x100)
            rows = b""
            for i in idx:
                if not tab["const"]:
                    rows += struct.pack(">I", tab["durations"][i])
                rows += struct.pack(">I", tab["sizes"][i])
                rows += struct.pack(">I", 0 if tab["sync"][i] else 0x00010000)
                rows += struct.pack(">i", tab["cto"][i])
            placements.append((len(trafs), len(payload)))
            trun_payload = struct.pack(">I", len(idx)) + b"\0\0\0\0" + rows  # data_offset patched below
            traf = (_full("tfhd", 0, 0x20000, struct.pack(">I", tab["id"])) +
                    _full("tfdt", 1, 0, struct.pack(">Q", dts[k])) +
                    _full("trun", 1, flags, trun_payload))
            trafs.append(traf)
            for i in idx:
                payload += b[tab["offsets"][i]:tab["offsets"][i] + tab["sizes"][i]]
                dts[k] += tab["durations"][i]
        mfhd = _full("mfhd", 0, 0, struct.pack(">I", seq))
        seq += 1
        moof_len = 8 + len(mfhd) + sum(8 + len(t) for t in trafs)
        # patch each trun's data_offset: moof start -> the traf's first sample in mdat
        fixed = []
        for (ti, poff), traf in zip(placements, trafs):
            data_offset = moof_len + 8 + poff
            at = traf.find(b"trun") + 4 + 4 + 4  # type, version/flags, sample_count
            traf = traf[:at] + struct.pack(">i", data_offset) + traf[at + 4:]
            fixed.append(_box("traf", traf))
        moof = _box("moof", mfhd + b"".join(fixed))
        assert len(moof) == moof_len
        out += moof + _box("mdat", bytes(payload))
    Path(dst).write_bytes(bytes(out))
    return {"tracks": tracks}
