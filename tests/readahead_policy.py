"""The read-ahead's window sizes (csrc/iris_api.hip, window_records), restated for the tests: a
walk from record 0 over `total` records in chunks of `chunk` computes its first chunk alone, then
windows of 2, 4, 8, ... chunks, at most 160 000 records (at least one chunk) and 64 MB of
[u16; 31] rows (window_chunks_max)."""

WINDOW_RECORDS = 160_000
ROWS_MAX = 64 << 20


def max_chunks(chunk, cap=None):
    w = cap if cap else max(1, WINDOW_RECORDS // chunk)
    return max(1, min(w, ROWS_MAX // (chunk * 31 * 2)))


def windows(total, chunk, cap=None):
    """Records of each read-ahead launch of one walk (a fresh engine) over [0, total)."""
    first = min(chunk, total)
    sizes, done = [first], first
    while done < total:
        w = min(2 * -(-sizes[-1] // chunk), max_chunks(chunk, cap))
        sizes.append(min(w * chunk, total - done))
        done += sizes[-1]
    return sizes


def counters(device):
    """(launches, records, largest window) of iris_config's readahead_windows."""
    return tuple(int(x) for x in device.config()["readahead_windows"].split("/"))
