"""LCM event-log reader/writer and the two message codecs the reference reads
(no ``lcm`` package needed).

Event framing (LCM log format): big-endian
  uint32 sync 0xEDA1DA01 | int64 event number | int64 timestamp (us) |
  int32 channel length | int32 data length | channel bytes | data bytes.
Messages (reference src/lcmtypes/lidar_t.py, odometry_t.py — generated LCM
code): an 8-byte fingerprint (the type hash rotated left by one bit), then
  lidar_t:    int64 utime, int32 n, float32 ranges[n], float32 thetas[n],
              int64 times[n], float32 intensities[n]
  odometry_t: int64 utime, float32 x, y, theta
Decoding is vectorised with NumPy big-endian dtypes (a log of ~10^5 scans
decodes in seconds instead of a per-field struct loop).
"""
import struct

import numpy as np

SYNC = 0xEDA1DA01


def _fingerprint(h):
    h &= 0xFFFFFFFFFFFFFFFF
    return struct.pack(">Q", ((h << 1) & 0xFFFFFFFFFFFFFFFF) + (h >> 63))


LIDAR_FP = _fingerprint(0xC4EE2DC3CD282B67)      # src/lcmtypes/lidar_t.py:59-63
ODOMETRY_FP = _fingerprint(0x0F98BD7892313B56)   # src/lcmtypes/odometry_t.py:49-53


def read_events(fname):
    """Yields (event_number, timestamp, channel, data bytes) in file order."""
    with open(fname, "rb") as f:
        buf = f.read()
    pos, n = 0, len(buf)
    while pos + 28 <= n:
        sync, num, ts, clen, dlen = struct.unpack_from(">IqqII", buf, pos)
        if sync != SYNC:
            raise ValueError(f"LCM log {fname}: bad sync word at byte {pos}")
        pos += 28
        if pos + clen + dlen > n:
            raise ValueError(f"LCM log {fname}: truncated event at byte {pos - 28}")
        channel = buf[pos:pos + clen].decode()
        pos += clen
        yield num, ts, channel, buf[pos:pos + dlen]
        pos += dlen


def write_events(fname, events):
    """events: iterable of (timestamp, channel, data bytes); numbered from 0."""
    with open(fname, "wb") as f:
        for num, (ts, channel, data) in enumerate(events):
            ch = channel.encode()
            f.write(struct.pack(">IqqII", SYNC, num, ts, len(ch), len(data)))
            f.write(ch)
            f.write(data)


def decode_lidar(data):
    """-> (utime, ranges float64 (n,), thetas float64 (n,)) — the float32
    fields widened exactly, as struct.unpack('>f') gives them."""
    if data[:8] != LIDAR_FP:
        raise ValueError("lidar_t decode error (fingerprint)")
    utime, n = struct.unpack_from(">qi", data, 8)
    o = 20
    ranges = np.frombuffer(data, dtype=">f4", count=n, offset=o).astype(np.float64)
    thetas = np.frombuffer(data, dtype=">f4", count=n, offset=o + 4 * n).astype(np.float64)
    return utime, ranges, thetas


def encode_lidar(utime, ranges, thetas, times=None, intensities=None):
    n = len(ranges)
    times = np.zeros(n, dtype=np.int64) if times is None else times
    intensities = np.zeros(n) if intensities is None else intensities
    return (LIDAR_FP + struct.pack(">qi", utime, n) + np.asarray(ranges, ">f4").tobytes() +
            np.asarray(thetas, ">f4").tobytes() + np.asarray(times, ">i8").tobytes() +
            np.asarray(intensities, ">f4").tobytes())


def decode_odometry(data):
    """-> (utime, x, y, theta) with the float32 fields widened exactly."""
    if data[:8] != ODOMETRY_FP:
        raise ValueError("odometry_t decode error (fingerprint)")
    return struct.unpack_from(">qfff", data, 8)


def encode_odometry(utime, x, y, theta):
    return ODOMETRY_FP + struct.pack(">qfff", utime, x, y, theta)
