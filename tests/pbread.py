"""A minimal protobuf wire reader for the tests (varint / length-delimited fields only)."""


def read_varint(b: bytes, i: int):
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x, i


def fields(b: bytes):
    """[(field number, wire type, value)] of one message; value = int (varint) or bytes (length-delimited)."""
    out, i = [], 0
    while i < len(b):
        key, i = read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = read_varint(b, i)
        elif wt == 2:
            n, i = read_varint(b, i)
            v, i = bytes(b[i:i + n]), i + n
        else:
            raise ValueError(f"wire type {wt}")
        out.append((num, wt, v))
    return out
