"""netCDF-4 (HDF5) quick-look files, from scratch.

The reference's published product (``QuickLook Data/CS2S3_<date>_25km_quicklook.nc``,
232 files; ``QuickLook Data/README.txt``) is netCDF-4: an HDF5 file (superblock
v0, version-2 object headers with compact links, HDF5 1.10.4 / netCDF 4.6.1)
holding ``lat``, ``lon``, ``radar_freeboard`` and ``uncertainty`` on a 320 x
320 grid of fp64, netCDF-4 dimension scales for the two dimensions, and CF-ish
attributes.  No HDF5 or netCDF library exists in this image, so this module
implements the subset of the HDF5 file format (HDF5 File Format Specification
version 3.0; the structures are listed where they are parsed) these files use:

* ``read(path)``  -> ``NcFile``: global attributes, dimensions (name, length,
  dimension-scale dataset), variables (dims, dtype, attributes, data) -- a
  netCDF-4 reader restricted to contiguous / compact datasets, fixed-size
  numeric and string types, scalar and simple dataspaces, compact link and
  attribute storage, object references and global-heap variable-length data
  (DIMENSION_LIST);
* ``write_quicklook(path, fs, sd, lat, lon, date, ...)`` writes the same layout
  (dimension scales, DIMENSION_LIST / REFERENCE_LIST / _Netcdf4Dimid /
  _Netcdf4Coordinates, the renamed ``_nc4_non_coord_lon`` dataset, fill values,
  Jenkins lookup3 checksums) as a netCDF-4 library would.

Only numpy is used.  ``tests/test_hdf5nc.py`` checks the reader against the
reference's own files (structure fixture in tests/golden/quicklook_layout.json)
and the writer by a round trip through the reader plus a layout comparison.
"""
import struct

import numpy as np

SIGNATURE = b'\x89HDF\r\n\x1a\n'
UNDEF = 0xFFFFFFFFFFFFFFFF


# ------------------------------------------------------------- checksum
def lookup3(data, initval=0):
    """Bob Jenkins' lookup3 ``hashlittle`` (the checksum of every HDF5 v2
    metadata block: H5_checksum_lookup3)."""
    def rot(x, k):
        return ((x << k) | (x >> (32 - k))) & 0xFFFFFFFF

    length = len(data)
    a = b = c = (0xDEADBEEF + length + initval) & 0xFFFFFFFF
    off = 0
    while length > 12:
        a = (a + int.from_bytes(data[off:off + 4], 'little')) & 0xFFFFFFFF
        b = (b + int.from_bytes(data[off + 4:off + 8], 'little')) & 0xFFFFFFFF
        c = (c + int.from_bytes(data[off + 8:off + 12], 'little')) & 0xFFFFFFFF
        a = (a - c) & 0xFFFFFFFF; a ^= rot(c, 4); c = (c + b) & 0xFFFFFFFF
        b = (b - a) & 0xFFFFFFFF; b ^= rot(a, 6); a = (a + c) & 0xFFFFFFFF
        c = (c - b) & 0xFFFFFFFF; c ^= rot(b, 8); b = (b + a) & 0xFFFFFFFF
        a = (a - c) & 0xFFFFFFFF; a ^= rot(c, 16); c = (c + b) & 0xFFFFFFFF
        b = (b - a) & 0xFFFFFFFF; b ^= rot(a, 19); a = (a + c) & 0xFFFFFFFF
        c = (c - b) & 0xFFFFFFFF; c ^= rot(b, 4); b = (b + a) & 0xFFFFFFFF
        off += 12
        length -= 12
    if length == 0:
        return c
    tail = data[off:] + b'\x00' * (12 - length)
    a = (a + int.from_bytes(tail[0:4], 'little')) & 0xFFFFFFFF
    b = (b + int.from_bytes(tail[4:8], 'little')) & 0xFFFFFFFF
    c = (c + int.from_bytes(tail[8:12], 'little')) & 0xFFFFFFFF
    c ^= b; c = (c - rot(b, 14)) & 0xFFFFFFFF
    a ^= c; a = (a - rot(c, 11)) & 0xFFFFFFFF
    b ^= a; b = (b - rot(a, 25)) & 0xFFFFFFFF
    c ^= b; c = (c - rot(b, 16)) & 0xFFFFFFFF
    a ^= c; a = (a - rot(c, 4)) & 0xFFFFFFFF
    b ^= a; b = (b - rot(a, 14)) & 0xFFFFFFFF
    c ^= b; c = (c - rot(b, 24)) & 0xFFFFFFFF
    return c


# ------------------------------------------------------------- datatypes
class Dtype:
    """An HDF5 datatype message (spec IV.A.2.d): class, size, and what the
    reader needs -- a numpy dtype for numeric classes, the base type of a
    variable-length sequence, the members of a compound."""

    def __init__(self, cls, version, bits, size, np_dtype=None, base=None, members=None, raw=b''):
        self.cls, self.version, self.bits, self.size = cls, version, bits, size
        self.np_dtype, self.base, self.members, self.raw = np_dtype, base, members, raw

    def describe(self):
        if self.cls in (0, 1):
            return str(self.np_dtype)
        if self.cls == 3:
            return f'string{self.size}'
        if self.cls == 7:
            return 'objref'
        if self.cls == 9:
            return f'vlen<{self.base.describe()}>'
        if self.cls == 6:
            return 'compound{' + ','.join(f'{n}:{t.describe()}@{o}' for n, o, t in self.members) + '}'
        return f'class{self.cls}'


def parse_dtype(buf, off):
    """-> (Dtype, bytes consumed)."""
    b0 = buf[off]
    cls, version = b0 & 0x0F, b0 >> 4
    bits = buf[off + 1] | (buf[off + 2] << 8) | (buf[off + 3] << 16)
    size = struct.unpack_from('<I', buf, off + 4)[0]
    p = off + 8
    if cls == 0:  # fixed point: bit offset, precision
        signed = bool(bits & 0x8)
        order = '>' if bits & 1 else '<'
        dt = np.dtype(f'{order}{"i" if signed else "u"}{size}')
        p += 4
        return Dtype(cls, version, bits, size, dt, raw=bytes(buf[off:p])), p - off
    if cls == 1:  # floating point: offset, precision, exp loc/size, mant loc/size, bias
        order = '>' if bits & 1 else '<'
        dt = np.dtype(f'{order}f{size}')
        p += 12
        return Dtype(cls, version, bits, size, dt, raw=bytes(buf[off:p])), p - off
    if cls in (3, 7):  # string (no properties), reference (version 1: none)
        return Dtype(cls, version, bits, size, raw=bytes(buf[off:p])), p - off
    if cls == 9:  # variable-length: base type follows
        base, nb = parse_dtype(buf, p)
        p += nb
        return Dtype(cls, version, bits, size, base=base, raw=bytes(buf[off:p])), p - off
    if cls == 6:  # compound, versions 1-3
        nmem = bits & 0xFFFF
        members = []
        for _ in range(nmem):
            e = buf.index(b'\x00', p)
            name = bytes(buf[p:e]).decode()
            if version < 3:   # name null-terminated, padded to a multiple of 8
                p += ((e + 1 - p + 7) // 8) * 8
            else:
                p = e + 1
            if version == 1:
                moff = struct.unpack_from('<I', buf, p)[0]
                p += 4 + 1 + 3 + 4 + 4 + 16  # offset, dimensionality, reserved, permutation, reserved, dims
            elif version == 2:
                moff = struct.unpack_from('<I', buf, p)[0]
                p += 4
            else:
                nbytes = max(1, (size.bit_length() + 7) // 8)
                moff = int.from_bytes(buf[p:p + nbytes], 'little')
                p += nbytes
            mt, nb = parse_dtype(buf, p)
            p += nb
            members.append((name, moff, mt))
        return Dtype(cls, version, bits, size, members=members, raw=bytes(buf[off:p])), p - off
    raise NotImplementedError(f'HDF5 datatype class {cls}')


def parse_dataspace(buf, off):
    """Dataspace message (spec IV.A.2.b), versions 1 and 2 -> shape tuple
    (() for scalar, None for null)."""
    version, rank, flags = buf[off], buf[off + 1], buf[off + 2]
    if version == 1:
        p = off + 8
        kind = 1 if rank else 0
    else:
        kind = buf[off + 3]
        p = off + 4
    dims = struct.unpack_from(f'<{rank}Q', buf, p) if rank else ()
    if kind == 2:
        return None
    return tuple(int(d) for d in dims)


# ------------------------------------------------------------- file model
class Variable:
    def __init__(self, name, dims, dtype, attrs, data, hdf5_name=None):
        self.name, self.dims, self.dtype, self.attrs, self.data = name, dims, dtype, attrs, data
        self.hdf5_name = hdf5_name or name


class NcFile:
    """What ``read`` returns: ``attrs`` (global), ``dims`` {name: length} in
    dimension-id order, ``variables`` {name: Variable}, and ``objects`` (the
    raw HDF5 view: {hdf5 name: {'attrs', 'shape', 'dtype', 'layout', 'messages'}})."""

    def __init__(self):
        self.attrs, self.dims, self.variables, self.objects = {}, {}, {}, {}
        self.superblock = {}


class _Reader:
    def __init__(self, buf):
        self.buf = buf
        self.heaps = {}

    # global heap collection (spec III.E): object index -> bytes
    def heap_object(self, addr, index):
        if addr not in self.heaps:
            b = self.buf
            assert b[addr:addr + 4] == b'GCOL', 'global heap signature'
            csize = struct.unpack_from('<Q', b, addr + 8)[0]
            objs, p, end = {}, addr + 16, addr + csize
            while p + 16 <= end:
                idx, _ref = struct.unpack_from('<HH', b, p)
                osize = struct.unpack_from('<Q', b, p + 8)[0]
                if idx == 0:
                    break
                objs[idx] = bytes(b[p + 16:p + 16 + osize])
                p += 16 + ((osize + 7) // 8) * 8
            self.heaps[addr] = objs
        return self.heaps[addr][index]

    def messages(self, addr):
        """All messages of the object header at ``addr`` (v1 or v2 with its
        continuation blocks, spec IV.A.1): [(type, flags, bytes)]."""
        b = self.buf
        out = []
        if b[addr:addr + 4] == b'OHDR':
            version, flags = b[addr + 4], b[addr + 5]
            assert version == 2
            p = addr + 6
            if flags & 0x20:
                p += 16
            if flags & 0x10:
                p += 4
            szb = 1 << (flags & 3)
            chunk = int.from_bytes(b[p:p + szb], 'little')
            p += szb
            blocks = [(p, p + chunk, addr)]
            co = 2 if flags & 0x04 else 0
            while blocks:
                start, end, block_addr = blocks.pop(0)
                # checksum of the block (signature .. end), stored after it
                stored = struct.unpack_from('<I', b, end)[0]
                if lookup3(bytes(b[block_addr:end])) != stored:
                    raise ValueError(f'object header checksum mismatch at {block_addr:#x}')
                q = start
                while q + 4 + co <= end:
                    mtype = b[q]
                    msize = struct.unpack_from('<H', b, q + 1)[0]
                    mflags = b[q + 3]
                    q += 4 + co
                    data = bytes(b[q:q + msize])
                    q += msize
                    if mtype == 0x10:  # continuation: OCHK block
                        caddr, clen = struct.unpack('<QQ', data[:16])
                        assert b[caddr:caddr + 4] == b'OCHK'
                        blocks.append((caddr + 4, caddr + clen - 4, caddr))
                    out.append((mtype, mflags, data))
            return out
        # version 1 header: version, reserved, nmesg(2), refcount(4), size(4), pad to 8
        version = b[addr]
        assert version == 1, f'unknown object header at {addr:#x}'
        nmesg = struct.unpack_from('<H', b, addr + 2)[0]
        size = struct.unpack_from('<I', b, addr + 8)[0]
        blocks = [(addr + 16, addr + 16 + size)]
        while blocks and len(out) < nmesg:
            q, end = blocks.pop(0)
            while q + 8 <= end and len(out) < nmesg:
                mtype, msize, mflags = struct.unpack_from('<HHB', b, q)
                data = bytes(b[q + 8:q + 8 + msize])
                q += 8 + msize
                if mtype == 0x10:
                    caddr, clen = struct.unpack('<QQ', data[:16])
                    blocks.append((caddr, caddr + clen))
                out.append((mtype, mflags, data))
        return out

    def attribute(self, data):
        """Attribute message (spec IV.A.2.m), versions 1 and 3 -> (name, value, Dtype, shape)."""
        version = data[0]
        name_sz, dt_sz, ds_sz = struct.unpack_from('<HHH', data, 2)
        if version == 1:
            p = 8
            pad = lambda n: ((n + 7) // 8) * 8
            name = data[p:p + name_sz].split(b'\x00')[0].decode()
            p += pad(name_sz)
            dt, _ = parse_dtype(data, p)
            p += pad(dt_sz)
            shape = parse_dataspace(data, p)
            p += pad(ds_sz)
        else:
            p = 9 if version == 3 else 8
            name = data[p:p + name_sz].split(b'\x00')[0].decode()
            p += name_sz
            dt, _ = parse_dtype(data, p)
            p += dt_sz
            shape = parse_dataspace(data, p)
            p += ds_sz
        return name, self.value(dt, shape, data, p), dt, shape

    def value(self, dt, shape, data, p):
        count = int(np.prod(shape)) if shape else 1
        if shape is None:
            return None
        if dt.cls == 3:
            s = data[p:p + dt.size].split(b'\x00')[0].decode('utf-8', errors='replace')
            return s
        if dt.cls in (0, 1):
            a = np.frombuffer(data, dtype=dt.np_dtype, count=count, offset=p).copy()
            return a.reshape(shape) if shape else a[0]
        if dt.cls == 7:
            return [struct.unpack_from('<Q', data, p + 8 * k)[0] for k in range(count)]
        if dt.cls == 9:  # each element: length (4), heap collection address (8), index (4)
            out = []
            for k in range(count):
                ln, haddr, hidx = struct.unpack_from('<IQI', data, p + 16 * k)
                raw = self.heap_object(haddr, hidx) if ln else b''
                if dt.base.cls == 7:
                    out.append([struct.unpack_from('<Q', raw, 8 * e)[0] for e in range(ln)])
                else:
                    out.append(np.frombuffer(raw, dtype=dt.base.np_dtype, count=ln).copy())
            return out
        if dt.cls == 6:
            out = []
            for k in range(count):
                rec = {}
                for mname, moff, mt in dt.members:
                    rec[mname] = self.value(mt, (), data, p + k * dt.size + moff)
                    if isinstance(rec[mname], list) and len(rec[mname]) == 1:
                        rec[mname] = rec[mname][0]
                out.append(rec)
            return out
        raise NotImplementedError(dt.describe())

    def obj(self, addr):
        """An object's links (group), attributes, and dataset messages."""
        o = {'addr': addr, 'attrs': {}, 'attr_types': {}, 'links': {}, 'shape': None, 'dtype': None,
             'layout': None, 'fill': None, 'message_types': []}
        for mtype, _mflags, data in self.messages(addr):
            o['message_types'].append(mtype)
            if mtype == 0x01:
                o['shape'] = parse_dataspace(data, 0)
            elif mtype == 0x03:
                o['dtype'], _ = parse_dtype(data, 0)
            elif mtype == 0x05:  # fill value v2/v3
                version, fl = data[0], data[1]
                if version == 3 and fl & 0x20:
                    sz = struct.unpack_from('<I', data, 2)[0]
                    o['fill'] = data[6:6 + sz]
                elif version == 2 and data[3]:
                    sz = struct.unpack_from('<I', data, 4)[0]
                    o['fill'] = data[8:8 + sz]
            elif mtype == 0x08:  # data layout v3 (spec IV.A.2.i)
                version, cls = data[0], data[1]
                assert version == 3
                if cls == 1:
                    a, n = struct.unpack_from('<QQ', data, 2)
                    o['layout'] = ('contiguous', a, n)
                elif cls == 0:
                    n = struct.unpack_from('<H', data, 2)[0]
                    o['layout'] = ('compact', data[4:4 + n])
                else:
                    o['layout'] = ('chunked',)
            elif mtype == 0x06:  # link (spec IV.A.2.g): hard links only
                version, fl = data[0], data[1]
                p = 2
                ltype = 0
                if fl & 0x08:
                    ltype = data[p]; p += 1
                if fl & 0x04:
                    p += 8
                if fl & 0x10:
                    p += 1
                nb = 1 << (fl & 3)
                ln = int.from_bytes(data[p:p + nb], 'little'); p += nb
                name = data[p:p + ln].decode(); p += ln
                if ltype == 0:
                    o['links'][name] = struct.unpack_from('<Q', data, p)[0]
            elif mtype == 0x0C:
                name, val, dt, shape = self.attribute(data)
                o['attrs'][name] = val
                o['attr_types'][name] = (dt.describe(), shape)
            elif mtype == 0x15:  # attribute info: dense storage not supported
                version, fl = data[0], data[1]
                p = 2 + (2 if fl & 1 else 0)
                fheap = struct.unpack_from('<Q', data, p)[0]
                if fheap != UNDEF:
                    raise NotImplementedError('dense attribute storage')
            elif mtype == 0x02:  # link info: dense link storage not supported
                fl = data[1]
                p = 2 + (8 if fl & 1 else 0)
                if struct.unpack_from('<Q', data, p)[0] != UNDEF:
                    raise NotImplementedError('dense link storage')
        return o

    def data(self, o):
        if o['layout'] is None or o['dtype'] is None or o['shape'] is None:
            return None
        n = int(np.prod(o['shape']))
        dt = o['dtype'].np_dtype
        if o['layout'][0] == 'contiguous':
            addr = o['layout'][1]
            if addr == UNDEF:  # never written: the fill value
                fill = np.frombuffer(o['fill'], dtype=dt)[0] if o['fill'] else 0
                return np.full(o['shape'], fill, dtype=dt)
            return np.frombuffer(self.buf, dtype=dt, count=n, offset=addr).reshape(o['shape']).copy()
        if o['layout'][0] == 'compact':
            return np.frombuffer(o['layout'][1], dtype=dt, count=n).reshape(o['shape']).copy()
        raise NotImplementedError('chunked datasets')


def read(path):
    """Parse a netCDF-4 file of the quick-look kind (see module docstring)."""
    buf = memoryview(open(path, 'rb').read())
    if bytes(buf[:8]) != SIGNATURE:
        raise ValueError('not an HDF5 file')
    sbv = buf[8]
    nc = NcFile()
    if sbv in (0, 1):  # superblock v0/1 (spec II.A): root symbol-table entry at 56 (v0)
        so, sl = buf[13], buf[14]
        assert so == 8 and sl == 8
        p = 24 + (4 if sbv == 1 else 0)
        base, _fs, eof, _drv = struct.unpack_from('<QQQQ', buf, p)
        root = struct.unpack_from('<Q', buf, p + 32 + 8)[0]
    else:  # v2/3: sizes, flags, base, ext, eof, root, checksum
        base, _ext, eof, root = struct.unpack_from('<QQQQ', buf, 12)
        if lookup3(bytes(buf[:44])) != struct.unpack_from('<I', buf, 44)[0]:
            raise ValueError('superblock checksum mismatch')
    nc.superblock = {'version': sbv, 'eof': eof, 'root': root}
    r = _Reader(buf)
    ro = r.obj(root)
    nc.attrs = {k: v for k, v in ro['attrs'].items()}
    nc.objects['/'] = ro
    objs = {}
    for name, addr in ro['links'].items():
        o = r.obj(addr)
        o['data'] = r.data(o)
        objs[name] = o
        nc.objects[name] = o
    # dimensions: dimension scales, ordered by _Netcdf4Dimid
    dims = []
    for name, o in objs.items():
        if o['attrs'].get('CLASS') == 'DIMENSION_SCALE':
            did = int(np.ravel(o['attrs'].get('_Netcdf4Dimid', len(dims)))[0])
            dims.append((did, name, int(o['shape'][0])))
    nc.dims = {n: ln for _, n, ln in sorted(dims)}
    dimscale_name = {o['addr']: n for n, o in objs.items() if o['attrs'].get('CLASS') == 'DIMENSION_SCALE'}
    for name, o in objs.items():
        nm = o['attrs'].get('NAME', '')
        if isinstance(nm, str) and nm.startswith('This is a netCDF dimension but not a netCDF variable'):
            continue  # a pure dimension
        vname = name[len('_nc4_non_coord_'):] if name.startswith('_nc4_non_coord_') else name
        if 'DIMENSION_LIST' in o['attrs']:
            vd = [dimscale_name[refs[0]] for refs in o['attrs']['DIMENSION_LIST']]
        elif o['attrs'].get('CLASS') == 'DIMENSION_SCALE':
            coords = o['attrs'].get('_Netcdf4Coordinates')
            if coords is not None:
                names = list(nc.dims)
                vd = [names[int(k)] for k in np.ravel(coords)]
            else:
                vd = [name]
        else:
            vd = []
        hidden = ('CLASS', 'NAME', 'REFERENCE_LIST', 'DIMENSION_LIST', '_Netcdf4Dimid', '_Netcdf4Coordinates')
        attrs = {k: v for k, v in o['attrs'].items() if k not in hidden}
        nc.variables[vname] = Variable(vname, vd, str(o['dtype'].np_dtype) if o['dtype'] else None, attrs,
                                       o['data'], hdf5_name=name)
    return nc


# ============================================================= writer
# Every message below is encoded as HDF5 1.10.4 under netCDF 4.6.1 encodes it in
# the reference's files (tests/test_hdf5nc.py compares them byte for byte, up to
# addresses): superblock v0, version-2 object headers with attribute creation
# order tracked + indexed (flags 0x0d), version-1 attribute / dataspace /
# datatype messages, contiguous layout v3, fill value messages 0x04 + 0x05 v2.
NC_FILL_DOUBLE = 9.969209968386869e36


def _dt_float64():
    # class 1 v1, little endian, implied-msb mantissa, sign bit 63; offset 0,
    # precision 64, exponent at 52 (11 bits), mantissa at 0 (52 bits), bias 1023
    return bytes([0x11, 0x20, 0x3F, 0x00]) + struct.pack('<I', 8) + struct.pack('<HHBBBBI', 0, 64, 52, 11, 0, 52, 1023)


def _dt_float32_be():
    # the netCDF-4 pure-dimension dataset type (H5T_IEEE_F32BE)
    return bytes([0x11, 0x21, 0x1F, 0x00]) + struct.pack('<I', 4) + struct.pack('<HHBBBBI', 0, 32, 23, 8, 0, 23, 127)


def _dt_int32():
    return bytes([0x10, 0x08, 0x00, 0x00]) + struct.pack('<I', 4) + struct.pack('<HH', 0, 32)


def _dt_string(n):
    return bytes([0x13, 0x00, 0x00, 0x00]) + struct.pack('<I', n)   # null-terminated ASCII


def _dt_objref():
    return bytes([0x17, 0x00, 0x00, 0x00]) + struct.pack('<I', 8)


def _dt_vlen_objref():
    return bytes([0x19, 0x00, 0x00, 0x00]) + struct.pack('<I', 16) + _dt_objref()


def _dt_reflist():
    """compound v1 {dataset: object reference @0, dimension: int32 @8}, size 16."""
    def member(name, off, dt):
        nm = name.encode() + b'\x00'
        nm += b'\x00' * ((-len(nm)) % 8)
        return nm + struct.pack('<IB3sII16s', off, 0, b'', 0, 0, b'') + dt
    body = member('dataset', 0, _dt_objref()) + member('dimension', 8, _dt_int32())
    return bytes([0x16, 0x02, 0x00, 0x00]) + struct.pack('<I', 16) + body


def _ds(dims):
    """Dataspace v1; scalar for dims == (), else simple with max dims = dims."""
    if not dims:
        return bytes([1, 0, 0, 0, 0, 0, 0, 0])
    return bytes([1, len(dims), 1, 0, 0, 0, 0, 0]) + struct.pack(f'<{2 * len(dims)}Q', *dims, *dims)


def _attr(name, dt, ds, data):
    """Attribute message v1: name, datatype and dataspace each padded to 8."""
    pad = lambda x: x + b'\x00' * ((-len(x)) % 8)
    nm = name.encode() + b'\x00'
    return bytes([1, 0]) + struct.pack('<HHH', len(nm), len(dt), len(ds)) + pad(nm) + pad(dt) + pad(ds) + data


def _attr_str(name, s):
    raw = s.encode() + (b'\x00' if name in ('_NCProperties', 'CLASS', 'NAME') else b'')
    return _attr(name, _dt_string(len(raw)), _ds(()), raw)


def _attr_i32(name, vals, scalar=False):
    v = np.atleast_1d(np.asarray(vals, dtype='<i4'))
    return _attr(name, _dt_int32(), _ds(() if scalar else (len(v),)), v.tobytes())


def _msg(mtype, data, flags=0, corder=0):
    return struct.pack('<BHBH', mtype, len(data), flags, corder) + data


def _ohdr(messages):
    """Version-2 object header: attribute creation order tracked and indexed
    (flags 0x0d: 2-byte chunk size), one chunk, lookup3 checksum."""
    body = b''.join(messages)
    blk = b'OHDR' + bytes([2, 0x0D]) + struct.pack('<H', len(body)) + body
    return blk + struct.pack('<I', lookup3(blk))


def _attr_info(max_corder):
    # attribute info v0, creation order tracked + indexed, compact storage
    return _msg(0x15, bytes([0, 0x03]) + struct.pack('<HQQQ', max_corder, UNDEF, UNDEF, UNDEF), flags=0x04)


def _dataset_header(shape, dt, fill, data_addr, nbytes, attrs):
    """Dataspace, datatype, fill values (old 0x04 + v2 0x05), contiguous layout,
    attribute info, then ``attrs`` [(creation order, encoded attribute)]."""
    msgs = [_msg(0x01, _ds(shape)), _msg(0x03, dt, flags=0x01)]
    if fill is not None:
        msgs.append(_msg(0x04, struct.pack('<I', len(fill)) + fill, flags=0x01))
    # fill value v2: allocation late (2), write time "if set" (2), defined
    msgs.append(_msg(0x05, bytes([2, 2, 2, 1]) + struct.pack('<I', len(fill) if fill else 0) + (fill or b''),
                     flags=0x01))
    msgs.append(_msg(0x08, bytes([3, 1]) + struct.pack('<QQ', data_addr, nbytes)))
    msgs.append(_attr_info(max(c for c, _ in attrs) + 1 if attrs else 0))
    msgs += [_msg(0x0C, a, corder=c) for c, a in attrs]
    return _ohdr(msgs)


def write_quicklook(path, fs, sd, lat, lon, date='20181201', created=None,
                    title=None, provenance='Gregory et al (UCL). https://doi.org/10.5194/tc-15-2857-2021'):
    """Write a quick-look day in the layout of the reference's
    ``QuickLook Data/CS2S3_<date>_25km_quicklook.nc`` (netCDF-4 / HDF5):
    dimensions ``lat`` (id 0) and ``lon`` (id 1); variables ``lat(lat, lon)``
    (the ``lat`` dimension scale itself, ``_Netcdf4Coordinates`` = [0, 1]),
    ``lon(lat, lon)`` (HDF5 dataset ``_nc4_non_coord_lon``: a pure ``lon``
    dimension scale holds the name), ``radar_freeboard(lat, lon)`` and
    ``uncertainty(lat, lon)``, fp64 with the reference's attributes and
    NC_FILL_DOUBLE fill values; global attributes _NCProperties, title,
    file_created_by, date_created, data_type.  ``fs`` / ``sd`` are the pass-2
    fields (``date+'_interp_smth'`` / ``'_interp_error_smth'``, GPR:333-334)
    on the grid, NaN where there is no output."""
    fs, sd, lat, lon = (np.ascontiguousarray(a, dtype='<f8') for a in (fs, sd, lat, lon))
    ny, nx = fs.shape
    for a in (sd, lat, lon):
        if a.shape != (ny, nx):
            raise ValueError('all fields must share the grid shape')
    title = title if title is not None else f'{date} CS2S3 radar freeboard and uncertainty'
    created = created if created is not None else date
    fill = np.array([NC_FILL_DOUBLE], dtype='<f8').tobytes()
    nbytes = ny * nx * 8
    order = ['lat', 'lon', '_nc4_non_coord_lon', 'radar_freeboard', 'uncertainty']  # link creation order
    users = ['_nc4_non_coord_lon', 'radar_freeboard', 'uncertainty']               # 2-D non-scale variables
    data_of = {'lat': lat, '_nc4_non_coord_lon': lon, 'radar_freeboard': fs, 'uncertainty': sd}

    def build(addr):
        """All metadata blocks for object addresses ``addr`` (sizes never depend on them)."""
        heap = []   # global heap objects: one object reference per DIMENSION_LIST entry

        def dimlist():
            ent = []
            for target in (addr['lat'], addr['lon']):
                heap.append(struct.pack('<Q', target))
                ent.append(struct.pack('<IQI', 1, addr['heap'], len(heap)))
            return _attr('DIMENSION_LIST', _dt_vlen_objref(), _ds((2,)), b''.join(ent))

        def reflist(dim):
            rec = b''.join(struct.pack('<Qi4x', addr[u], dim) for u in users)
            return _attr('REFERENCE_LIST', _dt_reflist(), _ds((len(users),)), rec)

        blk = {}
        blk['lat'] = _dataset_header((ny, nx), _dt_float64(), fill, addr['data:lat'], nbytes, [
            (0, _attr_str('CLASS', 'DIMENSION_SCALE')), (1, _attr_str('NAME', 'lat')),
            (2, _attr_i32('_Netcdf4Coordinates', [0, 1])), (3, _attr_i32('_Netcdf4Dimid', 0, scalar=True)),
            (4, _attr_str('units', 'degrees_north')), (5, _attr_str('long_name', 'latitude')),
            (6, reflist(0))])
        blk['lon'] = _dataset_header((nx,), _dt_float32_be(), None, UNDEF, nx * 4, [
            (0, _attr_str('CLASS', 'DIMENSION_SCALE')),
            (1, _attr_str('NAME', 'This is a netCDF dimension but not a netCDF variable.' + f'{nx:10d}')),
            (2, _attr_i32('_Netcdf4Dimid', 1, scalar=True)), (3, reflist(1))])
        for key, attrs in (('_nc4_non_coord_lon', [('units', 'degrees_east'), ('long_name', 'longitude')]),
                           ('radar_freeboard', [('units', 'metres'), ('standard_name', 'radar_freeboard')]),
                           ('uncertainty', [('units', 'metres'),
                                            ('standard_name', 'radar_freeboard_uncertainty')])):
            enc = [(k, _attr_str(a, v)) for k, (a, v) in enumerate(attrs)]
            enc += [(2, dimlist()), (3, _attr_i32('_Netcdf4Dimid', 0, scalar=True))]
            blk[key] = _dataset_header((ny, nx), _dt_float64(), fill, addr['data:' + key], nbytes, enc)
        # root group: link info (creation order tracked + indexed, compact), group info,
        # attribute info, the global attributes, one hard link per dataset
        glob = [_attr_str('_NCProperties', 'version=1|netcdflibversion=4.6.1|hdf5libversion=1.10.4'),
                _attr_str('title', title), _attr_str('file_created_by', provenance),
                _attr_str('date_created', created), _attr_str('data_type', 'Quick Look')]
        msgs = [_msg(0x02, bytes([0, 0x03]) + struct.pack('<QQQ', len(order), UNDEF, UNDEF) + struct.pack('<Q', UNDEF)),
                _msg(0x0A, bytes([0, 0]), flags=0x01)]
        msgs += [_msg(0x0C, a, corder=k) for k, a in enumerate(glob)]
        msgs.append(_attr_info(len(glob)))
        for k, name in enumerate(order):
            nm = name.encode()
            msgs.append(_msg(0x06, bytes([1, 0x04]) + struct.pack('<Q', k) + bytes([len(nm)]) + nm
                             + struct.pack('<Q', addr[name])))
        blk['/'] = _ohdr(msgs)
        # global heap collection (>= 4 KiB): objects, then the free-space object 0
        g = bytearray()
        for idx, o in enumerate(heap, 1):
            g += struct.pack('<HHIQ', idx, 0, 0, len(o)) + o + b'\x00' * ((-len(o)) % 8)
        size = max(4096, 16 + len(g) + 16)
        free = size - 16 - len(g)
        blk['heap'] = b'GCOL' + bytes([1, 0, 0, 0]) + struct.pack('<Q', size) + bytes(g) + \
            struct.pack('<HHIQ', 0, 0, 0, free) + b'\x00' * (free - 16)
        return blk

    # pass 1 sizes; pass 2 with the addresses: superblock | root | datasets | heap | data
    zero = {k: 0 for k in order + ['heap'] + ['data:' + k for k in data_of]}
    sizes = {k: len(v) for k, v in build(zero).items()}
    addr, pos = {}, 96
    for k in ['/'] + order + ['heap']:
        addr[k] = pos
        pos += sizes[k]
    pos = (pos + 7) // 8 * 8
    for k in ['lat', '_nc4_non_coord_lon', 'radar_freeboard', 'uncertainty']:
        addr['data:' + k] = pos
        pos += nbytes
    blk = build(addr)
    img = bytearray()
    sb = SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack('<HHI', 4, 16, 0)
    sb += struct.pack('<QQQQ', 0, UNDEF, pos, UNDEF)
    sb += struct.pack('<QQII16s', 0, addr['/'], 0, 0, b'')  # root symbol table entry (no cache)
    img += sb
    for k in ['/'] + order + ['heap']:
        assert len(img) == addr[k] and len(blk[k]) == sizes[k]
        img += blk[k]
    img += b'\x00' * (addr['data:lat'] - len(img))
    for k in ['lat', '_nc4_non_coord_lon', 'radar_freeboard', 'uncertainty']:
        img += data_of[k].tobytes()
    assert len(img) == pos
    with open(path, 'wb') as fh:
        fh.write(img)
    return path
