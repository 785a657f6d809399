"""The from-scratch netCDF-4 / HDF5 quick-look I/O (optimalinterpolation_amd/
hdf5nc.py) against the reference's published product
(``QuickLook Data/CS2S3_<date>_25km_quicklook.nc``, 232 files).

The layout fixture (tests/golden/quicklook_layout.json, made by
tests/golden/make_quicklook_layout.py from the reference's files) holds what
the files contain; where /root/reference is present the files themselves are
parsed too.  The writer must reproduce the reference's objects, attributes,
types and every address-free message byte for byte."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from optimalinterpolation_amd import day, hdf5nc

REF_DIR = '/root/reference/QuickLook Data'
HAVE_REF = os.path.isdir(REF_DIR)


def fixture():
    with open(os.path.join(GOLDEN, 'quicklook_layout.json')) as f:
        return json.load(f)


def test_lookup3_known_answers():
    # lookup3.c's own self-test values (driver5: hashlittle of these strings)
    assert hdf5nc.lookup3(b'') == 0xDEADBEEF
    assert hdf5nc.lookup3(b'Four score and seven years ago') == 0x17770551
    assert hdf5nc.lookup3(b'Four score and seven years ago', 1) == 0xCD628161


@pytest.mark.skipif(not HAVE_REF, reason='reference files absent (GPU box)')
def test_reads_reference_files():
    fx = fixture()
    names = sorted(fx['per_file'])
    for name in names[::29] + [names[-1]]:          # 9 days spread over the season
        nc = hdf5nc.read(os.path.join(REF_DIR, name))
        assert nc.attrs == fx['per_file'][name]['attrs']
        assert nc.dims == fx['per_file'][name]['dims']
        assert set(nc.variables) == {'lat', 'lon', 'radar_freeboard', 'uncertainty'}
        for v in nc.variables.values():
            assert v.dims == ['lat', 'lon'] and v.data.shape == (320, 320) and v.data.dtype == np.float64
    nc = hdf5nc.read(os.path.join(REF_DIR, fx['source']))
    for n, v in nc.variables.items():
        want = fx['layout']['variables'][n]
        assert hashlib.sha256(np.ascontiguousarray(v.data).tobytes()).hexdigest() == want['sha256']
        assert v.attrs == want['attrs']


def test_corrupt_checksum_is_rejected(tmp_path):
    p = str(tmp_path / 'q.nc')
    z = np.zeros((4, 5))
    hdf5nc.write_quicklook(p, z, z, z, z)
    b = bytearray(open(p, 'rb').read())
    k = b.index(b'OHDR', 200) + 20
    b[k] ^= 0x40
    open(p, 'wb').write(bytes(b))
    with pytest.raises(ValueError, match='checksum'):
        hdf5nc.read(p)


def _reference_like_fields(rng, shape=(320, 320)):
    lat = np.linspace(36.3, 89.9, shape[0] * shape[1]).reshape(shape)
    lon = np.linspace(-179.8, 179.9, shape[0] * shape[1]).reshape(shape)[::-1]
    fs = rng.normal(0.2, 0.1, shape)
    sd = np.abs(rng.normal(0.05, 0.02, shape))
    mask = rng.random(shape) < 0.85
    fs[mask] = np.nan
    sd[mask] = np.nan
    return fs, sd, lat, lon


def test_writer_round_trip(tmp_path):
    rng = np.random.default_rng(3)
    fs, sd, lat, lon = _reference_like_fields(rng, (37, 53))
    p = str(tmp_path / 'q.nc')
    hdf5nc.write_quicklook(p, fs, sd, lat, lon, date='20190101', created='20261017')
    nc = hdf5nc.read(p)
    assert nc.dims == {'lat': 37, 'lon': 53}
    assert nc.attrs['title'] == '20190101 CS2S3 radar freeboard and uncertainty'
    assert nc.attrs['date_created'] == '20261017'
    for n, a in (('radar_freeboard', fs), ('uncertainty', sd), ('lat', lat), ('lon', lon)):
        assert nc.variables[n].dims == ['lat', 'lon']
        assert np.array_equal(nc.variables[n].data, a, equal_nan=True)


def test_writer_layout_matches_reference(tmp_path):
    """Same objects, attribute names / types / shapes / values, dataset
    types, shapes, fill values and layouts as the reference file, and every
    address-free message identical byte for byte."""
    fx = fixture()
    lay = fx['layout']
    rng = np.random.default_rng(5)
    fs, sd, lat, lon = _reference_like_fields(rng)
    src = fx['source']
    date = src.split('_')[1]
    p = str(tmp_path / src)
    hdf5nc.write_quicklook(p, fs, sd, lat, lon, date=date, created=lay['attrs']['date_created'])
    nc = hdf5nc.read(p)
    assert nc.attrs == lay['attrs'] and nc.dims == lay['dims']
    assert set(nc.objects) == set(lay['objects'])
    for name, o in nc.objects.items():
        want = lay['objects'][name]
        assert (list(o['shape']) if o['shape'] is not None else None) == want['shape'], name
        assert (o['dtype'].describe() if o['dtype'] else None) == want['dtype'], name
        assert (o['layout'][0] if o['layout'] else None) == want['layout'], name
        assert (o['fill'].hex() if o['fill'] is not None else None) == want['fill'], name
        assert set(o['attrs']) == set(want['attrs']), name
        for k, v in o['attrs'].items():
            t, shape = o['attr_types'][k]
            assert t == want['attrs'][k]['type'] and list(shape) == want['attrs'][k]['shape'], (name, k)
            if want['attrs'][k]['value'] is not None:
                got = v.tolist() if isinstance(v, np.ndarray) else v.item() if isinstance(v, np.generic) else v
                assert got == want['attrs'][k]['value'], (name, k)
    for n, v in nc.variables.items():
        w = lay['variables'][n]
        assert v.dims == w['dims'] and v.dtype == w['dtype'] and v.hdf5_name == w['hdf5_name'] and v.attrs == w['attrs']
    # address-free messages, byte for byte
    import sys
    sys.path.insert(0, GOLDEN)
    from make_quicklook_layout import static_messages
    assert static_messages(p) == fx['static_messages']
    # the references resolve: DIMENSION_LIST -> the lat / lon scales, REFERENCE_LIST -> the users
    addr = {n: o['addr'] for n, o in nc.objects.items()}
    for n in ('_nc4_non_coord_lon', 'radar_freeboard', 'uncertainty'):
        assert nc.objects[n]['attrs']['DIMENSION_LIST'] == [[addr['lat']], [addr['lon']]]
    for d, n in enumerate(('lat', 'lon')):
        refs = nc.objects[n]['attrs']['REFERENCE_LIST']
        assert [r['dataset'] for r in refs][-3:] == [addr['_nc4_non_coord_lon'], addr['radar_freeboard'],
                                                     addr['uncertainty']]
        assert all(int(r['dimension']) == d for r in refs)


@pytest.mark.skipif(not HAVE_REF, reason='reference files absent (GPU box)')
def test_rewrite_reference_day_identical_content(tmp_path):
    """The reference's own day written back by the writer: every variable's
    data and attributes, the global attributes and dimensions identical."""
    fx = fixture()
    ref = hdf5nc.read(os.path.join(REF_DIR, fx['source']))
    v = ref.variables
    p = str(tmp_path / 'rewrite.nc')
    hdf5nc.write_quicklook(p, v['radar_freeboard'].data, v['uncertainty'].data, v['lat'].data, v['lon'].data,
                           date=fx['source'].split('_')[1], created=ref.attrs['date_created'])
    got = hdf5nc.read(p)
    assert got.attrs == ref.attrs and got.dims == ref.dims
    for n in ref.variables:
        assert np.array_equal(got.variables[n].data, v[n].data, equal_nan=True)
        assert got.variables[n].attrs == v[n].attrs and got.variables[n].dims == v[n].dims
    assert os.path.getsize(p) == os.path.getsize(os.path.join(REF_DIR, fx['source'])) - 688  # no OCHK / NIL slack


def test_day_write_quicklook_netcdf4(tmp_path):
    rng = np.random.default_rng(9)
    fs, sd, lat, lon = _reference_like_fields(rng, (16, 16))
    p = str(tmp_path / 'd.nc')
    day.write_quicklook(p, fs, sd, lat=lat, lon=lon, date='20181205')
    nc = hdf5nc.read(p)
    assert np.array_equal(nc.variables['uncertainty'].data, sd, equal_nan=True)
