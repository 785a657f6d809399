"""The layout of the reference's published quick-look files
(``/root/reference/QuickLook Data/CS2S3_<date>_25km_quicklook.nc``) as a
small JSON fixture, for tests/test_hdf5nc.py to check the from-scratch
netCDF-4 writer against where the reference is absent (the GPU box).

Run in the build container only (it reads /root/reference):
    python tests/golden/make_quicklook_layout.py

Parsed with optimalinterpolation_amd/hdf5nc.py's reader, which verifies every
object-header checksum of the file.  Recorded per HDF5 object: its attribute
names, types, shapes and values (strings / integers), the bytes of every
message that carries no file address (dataspace, datatype, fill values,
attributes other than DIMENSION_LIST / REFERENCE_LIST), and per variable a
digest of its data; plus the global attributes and dimensions of every file
(232 days: which attributes vary between files).  Data files only -- no
reference source is copied."""
import glob
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from optimalinterpolation_amd import hdf5nc  # noqa: E402

REF_DIR = '/root/reference/QuickLook Data'


def static_messages(path):
    """{object: sorted hex of its address-free messages}."""
    buf = memoryview(open(path, 'rb').read())
    r = hdf5nc._Reader(buf)
    nc = hdf5nc.read(path)
    out = {}
    for name, o in nc.objects.items():
        keep = []
        for mtype, _fl, data in r.messages(o['addr']):
            if mtype in (0x00, 0x10, 0x02, 0x06, 0x08, 0x15):   # NIL, continuation, links, layout, attr info
                continue
            if mtype == 0x0C:
                nlen = int.from_bytes(data[2:4], 'little')
                aname = bytes(data[8:8 + nlen - 1]).decode()
                if aname in ('DIMENSION_LIST', 'REFERENCE_LIST'):
                    continue
            keep.append(f'{mtype:02x}:' + data.hex())
        out[name] = sorted(keep)
    return out


def layout(path, with_data=True):
    nc = hdf5nc.read(path)
    objs = {}
    for name, o in nc.objects.items():
        attrs = {}
        for k, v in o['attrs'].items():
            t, shape = o['attr_types'][k]
            if isinstance(v, np.ndarray):
                v = v.tolist()
            elif isinstance(v, (np.integer, np.floating)):
                v = v.item()
            elif k in ('DIMENSION_LIST', 'REFERENCE_LIST'):
                v = None   # file addresses
            attrs[k] = {'type': t, 'shape': list(shape) if shape is not None else None, 'value': v}
        objs[name] = {'attrs': attrs, 'shape': list(o['shape']) if o['shape'] is not None else None,
                      'dtype': o['dtype'].describe() if o['dtype'] else None,
                      'layout': o['layout'][0] if o['layout'] else None,
                      'fill': o['fill'].hex() if o['fill'] is not None else None}
    var = {}
    for n, v in nc.variables.items():
        d = {'dims': v.dims, 'dtype': v.dtype, 'hdf5_name': v.hdf5_name, 'attrs': v.attrs}
        if with_data and v.data is not None:
            a = np.ascontiguousarray(v.data)
            d['sha256'] = hashlib.sha256(a.tobytes()).hexdigest()
            d['nan'] = int(np.isnan(a).sum())
            d['sample'] = [float(x) for x in a.ravel()[::10007]]
        var[n] = d
    return {'attrs': nc.attrs, 'dims': nc.dims, 'objects': objs, 'variables': var}


def main():
    files = sorted(glob.glob(os.path.join(REF_DIR, '*_quicklook.nc')))
    first = files[0]
    fixture = {'source': os.path.basename(first), 'n_files': len(files),
               'layout': layout(first), 'static_messages': static_messages(first),
               'per_file': {}}
    for f in files:
        lay = layout(f, with_data=False)
        fixture['per_file'][os.path.basename(f)] = {'attrs': lay['attrs'], 'dims': lay['dims'],
                                                    'size': os.path.getsize(f)}
    with open(os.path.join(HERE, 'quicklook_layout.json'), 'w') as fh:
        json.dump(fixture, fh, indent=1, sort_keys=True)
    print(f"{len(files)} files; fixture from {os.path.basename(first)}")


if __name__ == '__main__':
    main()
