"""The read-ahead's window sizes (csrc/iris_api.hip, window_records), restated for the tests: a
walk from record 0 over `total` records in chunks of `chunk` computes its first chunk alone, then
windows of 2, 4, 8, ... chunks, at most 64 MB of [u16; 31] rows (window_chunks_max) and at most
half of the chunks left (at least one)."""

ROWS_MAX = 64 << 20


def max_chunks(chunk):
    return max(1, ROWS_MAX // (chunk * 31 * 2))


def windows(total, chunk):
    """Records of each read-ahead launch of one walk (a fresh engine) over [0, total)."""
    first = min(chunk, total)
    sizes, done = [first], first
    while done < total:
        avail = total - done
        left = -(-avail // chunk)
        w = min(2 * -(-sizes[-1] // chunk), max(1, (left + 1) // 2), max_chunks(chunk))
        sizes.append(min(w * chunk, avail))
        done += sizes[-1]
    return sizes


def counters(device):
    """(launches, records, largest window) of iris_config's readahead_windows."""
    return tuple(int(x) for x in device.config()["readahead_windows"].split("/"))
