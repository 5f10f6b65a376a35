"""go_json.py -- CPU restatement of the reference's job/group ingestion, for
small inputs.  TEST INFRASTRUCTURE ONLY: imported by tests/ (never by the
product, which decodes in C++: cronsun_amd/csrc/cg_ingest.cpp).

Restates, in plain Python written from the Go sources' documented behaviour:
  * Go 1.7/1.8 encoding/json (the reference's CI Go versions, .travis.yml):
    scanner validity (checkValid), string unquoting (escapes, surrogate pairs,
    utf8.DecodeRune + U+FFFD for invalid bytes), object key -> field matching
    (exact, else fold.go's case folding incl. K/ſ), literalStore (null is a
    no-op for scalars and nil for slices/pointers, ParseInt for ints, type
    errors), array decoding into an existing slice (element reuse, growth to
    cap + cap/2 >= 4, truncation, empty -> new empty slice);
  * GetJobs (job.go:339-365): Unmarshal, Job.Valid (job.go:633-655,
    JobRule.Valid job.go:291-308: ErrNilRule, cron.Parse via the C oracle;
    a nil rule panics), alone() (job.go:378-382), last value per ID wins;
  * GetGroups("") (group.go:39-63): Unmarshal, last value per ID wins.
Parity pins: the reference has no JSON fixtures for jobs; the cases in
tests/test_ingest.py are derived from encoding/json's documented rules, so
this restatement is "parity unpinned" beyond them.
"""

OK, UNMARSHAL, INVALID, PANIC, REPLACED, UNSUPPORTED = 0, 1, 2, 3, 4, 5


class _Syntax(Exception):
    pass


# ----------------------------------------------------------------- scanner
_WS = b" \t\n\r"


def _ws(b, i):
    while i < len(b) and b[i] in _WS:
        i += 1
    return i


def _decode_rune(b, i, end):
    """utf8.DecodeRune on b[i:end] -> (rune, size); (0xFFFD, 1) if invalid."""
    c = b[i]
    if c < 0x80:
        return c, 1
    if 0xC2 <= c <= 0xDF:
        n, v, lo, hi = 2, c & 0x1F, 0x80, 0xBF
    elif 0xE0 <= c <= 0xEF:
        n, v = 3, c & 0x0F
        lo = 0xA0 if c == 0xE0 else 0x80
        hi = 0x9F if c == 0xED else 0xBF
    elif 0xF0 <= c <= 0xF4:
        n, v = 4, c & 0x07
        lo = 0x90 if c == 0xF0 else 0x80
        hi = 0x8F if c == 0xF4 else 0xBF
    else:
        return 0xFFFD, 1
    if end - i < n:
        return 0xFFFD, 1
    for k in range(1, n):
        x = b[i + k]
        if not ((lo if k == 1 else 0x80) <= x <= (hi if k == 1 else 0xBF)):
            return 0xFFFD, 1
        v = (v << 6) | (x & 0x3F)
    return v, n


def _hex4(b, i):
    if i + 4 > len(b):
        return -1
    try:
        s = b[i:i + 4].decode("ascii")
        if not all(ch in "0123456789abcdefABCDEF" for ch in s):
            return -1
        return int(s, 16)
    except UnicodeDecodeError:
        return -1


def _string(b, i):
    """b[i] == '"' -> (bytes value (UTF-8), next index)."""
    assert b[i] == 0x22
    i += 1
    j = i
    # find the closing quote, validating the body
    while True:
        if j >= len(b):
            raise _Syntax()
        c = b[j]
        if c == 0x22:
            break
        if c < 0x20:
            raise _Syntax()
        if c == 0x5C:
            if j + 1 >= len(b):
                raise _Syntax()
            k = b[j + 1]
            if k in b'"\\/bfnrt':
                j += 2
            elif k == 0x75:
                if _hex4(b, j + 2) < 0:
                    raise _Syntax()
                j += 6
            else:
                raise _Syntax()
        else:
            j += 1
    body, end = b[i:j], j + 1
    out = []
    r = 0
    esc = {0x22: 0x22, 0x5C: 0x5C, 0x2F: 0x2F, 0x62: 8, 0x66: 12, 0x6E: 10, 0x72: 13, 0x74: 9}
    while r < len(body):
        c = body[r]
        if c == 0x5C:
            k = body[r + 1]
            if k != 0x75:
                out.append(chr(esc[k]))
                r += 2
                continue
            rr = _hex4(body, r + 2)
            r += 6
            if 0xD800 <= rr < 0xE000:
                rr1 = _hex4(body, r + 2) if r + 1 < len(body) and body[r] == 0x5C and body[r + 1] == 0x75 else -1
                if rr < 0xDC00 and 0xDC00 <= rr1 < 0xE000:
                    out.append(chr(0x10000 + ((rr - 0xD800) << 10) + (rr1 - 0xDC00)))
                    r += 6
                    continue
                rr = 0xFFFD
            out.append(chr(rr))
            continue
        if c < 0x80:
            out.append(chr(c))
            r += 1
            continue
        rune, n = _decode_rune(body, r, len(body))
        out.append(chr(rune))
        r += n
    return "".join(out).encode("utf-8", "surrogatepass"), end


def _number(b, i):
    j = i
    if j < len(b) and b[j] == 0x2D:
        j += 1
    if j >= len(b):
        raise _Syntax()
    if b[j] == 0x30:
        j += 1
    elif 0x31 <= b[j] <= 0x39:
        while j < len(b) and 0x30 <= b[j] <= 0x39:
            j += 1
    else:
        raise _Syntax()
    if j < len(b) and b[j] == 0x2E:
        j += 1
        if j >= len(b) or not 0x30 <= b[j] <= 0x39:
            raise _Syntax()
        while j < len(b) and 0x30 <= b[j] <= 0x39:
            j += 1
    if j < len(b) and b[j] in b"eE":
        j += 1
        if j < len(b) and b[j] in b"+-":
            j += 1
        if j >= len(b) or not 0x30 <= b[j] <= 0x39:
            raise _Syntax()
        while j < len(b) and 0x30 <= b[j] <= 0x39:
            j += 1
    return b[i:j], j


def _value(b, i, depth=0):
    """-> (node, next index).  node: ('obj', [(key, node)]), ('arr', [node]),
    ('str', bytes), ('num', literal), ('bool', v), ('null',)."""
    if depth > 10000:
        raise _Syntax()
    i = _ws(b, i)
    if i >= len(b):
        raise _Syntax()
    c = b[i]
    if c == 0x7B:
        i = _ws(b, i + 1)
        pairs = []
        if i < len(b) and b[i] == 0x7D:
            return ("obj", pairs), i + 1
        while True:
            i = _ws(b, i)
            if i >= len(b) or b[i] != 0x22:
                raise _Syntax()
            k, i = _string(b, i)
            i = _ws(b, i)
            if i >= len(b) or b[i] != 0x3A:
                raise _Syntax()
            v, i = _value(b, i + 1, depth + 1)
            pairs.append((k, v))
            i = _ws(b, i)
            if i < len(b) and b[i] == 0x2C:
                i += 1
                continue
            if i < len(b) and b[i] == 0x7D:
                return ("obj", pairs), i + 1
            raise _Syntax()
    if c == 0x5B:
        i = _ws(b, i + 1)
        items = []
        if i < len(b) and b[i] == 0x5D:
            return ("arr", items), i + 1
        while True:
            v, i = _value(b, i, depth + 1)
            items.append(v)
            i = _ws(b, i)
            if i < len(b) and b[i] == 0x2C:
                i += 1
                continue
            if i < len(b) and b[i] == 0x5D:
                return ("arr", items), i + 1
            raise _Syntax()
    if c == 0x22:
        s, i = _string(b, i)
        return ("str", s), i
    for lit, node in ((b"true", ("bool", True)), (b"false", ("bool", False)), (b"null", ("null",))):
        if b.startswith(lit, i):
            return node, i + len(lit)
        if c == lit[0]:
            raise _Syntax()
    lit, i = _number(b, i)
    return ("num", lit), i


# ---------------------------------------------------------- field matching
def _fold_match(key, name):
    """fold.go (Go 1.8): the equalFold of field `name` (ASCII) against key."""
    special = any(ch in "kKsS" for ch in name)
    nb = name.encode()
    t = key
    if not special:
        if len(t) != len(nb):
            return False
        for sb, tb in zip(nb, t):
            if sb == tb:
                continue
            if (0x41 <= sb <= 0x5A or 0x61 <= sb <= 0x7A) and (sb & 0xDF) == (tb & 0xDF):
                continue
            return False
        return True
    for sb in nb:
        if not t:
            return False
        tb = t[0]
        if tb < 0x80:
            if sb != tb:
                su = sb & 0xDF
                if not (0x41 <= su <= 0x5A) or su != (tb & 0xDF):
                    return False
            t = t[1:]
            continue
        if sb in b"kK" and t.startswith(b"\xe2\x84\xaa"):
            t = t[3:]
            continue
        if sb in b"sS" and t.startswith(b"\xc5\xbf"):
            t = t[2:]
            continue
        return False
    return len(t) == 0


def _field(key, names):
    for n in names:
        if key == n.encode():
            return n
    for n in names:
        if _fold_match(key, n):
            return n
    return None


# ------------------------------------------------------------- decoding
class _TypeErr(Exception):
    pass


class GoSlice:
    def __init__(self):
        self.backing, self.len = [], 0

    def items(self):
        return self.backing[:self.len]


def _store_string(node, cur):
    if node[0] == "null":
        return cur
    if node[0] != "str":
        raise _TypeErr()
    return node[1]


def _store_int(node, cur):
    if node[0] == "null":
        return cur
    if node[0] != "num":
        raise _TypeErr()
    s = node[1]
    digits = s[1:] if s.startswith(b"-") else s
    if not digits or not digits.isdigit():
        raise _TypeErr()
    v = int(s)
    if not -(1 << 63) <= v <= (1 << 63) - 1:
        raise _TypeErr()
    return v


def _store_bool(node, cur):
    if node[0] == "null":
        return cur
    if node[0] != "bool":
        raise _TypeErr()
    return node[1]


def _store_slice(node, sl, elem, zero):
    """decode.go array(): element reuse, growth, truncation."""
    if node[0] == "null":
        return GoSlice()
    if node[0] != "arr":
        raise _TypeErr()
    i = 0
    for item in node[1]:
        if i >= len(sl.backing):
            cap = len(sl.backing)
            nc = max(cap + cap // 2, 4)
            nb = [zero() for _ in range(nc)]
            nb[:sl.len] = sl.backing[:sl.len]
            sl.backing = nb
        if i >= sl.len:
            sl.len = i + 1
        sl.backing[i] = elem(item, sl.backing[i])
        i += 1
    if i < sl.len:
        sl.len = i
    if i == 0:
        sl = GoSlice()
    return sl


RULE_FIELDS = ["id", "timer", "gids", "nids", "exclude_nids"]
JOB_FIELDS = ["id", "name", "group", "cmd", "user", "rules", "pause", "timeout", "parallels",
              "retry", "interval", "kind", "avg_time", "fail_notify", "to"]
GROUP_FIELDS = ["id", "name", "nids"]


def _strings(node, sl):
    return _store_slice(node, sl, _store_string, lambda: b"")


def _decode_struct(node, obj, names, setter):
    if node[0] == "null":
        return obj
    if node[0] != "obj":
        raise _TypeErr()
    for k, v in node[1]:
        f = _field(k, names)
        if f is not None:
            setter(obj, f, v)
    return obj


def _new_rule():
    return {"id": b"", "timer": b"", "gids": GoSlice(), "nids": GoSlice(), "exclude_nids": GoSlice()}


def _set_rule(r, f, v):
    if f in ("id", "timer"):
        r[f] = _store_string(v, r[f])
    else:
        r[f] = _strings(v, r[f])


def _rule_elem(node, cur):
    if node[0] == "null":
        return None
    if node[0] != "obj":
        raise _TypeErr()
    r = cur if cur is not None else _new_rule()
    return _decode_struct(node, r, RULE_FIELDS, _set_rule)


def _set_job(j, f, v):
    if f in ("id", "name", "group", "cmd", "user"):
        j[f] = _store_string(v, j[f])
    elif f == "rules":
        j[f] = _store_slice(v, j[f], _rule_elem, lambda: None)
    elif f in ("pause", "fail_notify"):
        j[f] = _store_bool(v, j[f])
    elif f == "to":
        j[f] = _strings(v, j[f])
    else:
        j[f] = _store_int(v, j[f])


def _new_job():
    j = {f: b"" for f in ("id", "name", "group", "cmd", "user")}
    j.update({"rules": GoSlice(), "pause": False, "fail_notify": False, "to": GoSlice()})
    j.update({f: 0 for f in ("timeout", "parallels", "retry", "interval", "kind", "avg_time")})
    return j


def _unmarshal(doc, new, names, setter):
    """json.Unmarshal: (True, value) or (False, None)."""
    try:
        node, i = _value(doc, 0)
        if _ws(doc, i) != len(doc):
            raise _Syntax()
    except (_Syntax, IndexError):
        return False, None
    v = new()
    try:
        # a type error is recorded and decoding continues in Go; the value is
        # then discarded by GetJobs / GetGroups either way
        _decode_struct(node, v, names, setter)
    except _TypeErr:
        return False, None
    return True, v


def ingest_jobs(docs, parse):
    """GetJobs over `docs` (bytes).  parse(timer_bytes) -> schedule or None.
    Returns (status list, [(doc index, job dict with 'schedules')]) in the
    order the product adds them (doc order of each ID's last valid value)."""
    st, jobs = [], []
    for d in docs:
        ok, j = _unmarshal(d, _new_job, JOB_FIELDS, _set_job)
        if not ok:
            st.append(UNMARSHAL)
            jobs.append(None)
            continue
        status, scheds = OK, []
        for r in j["rules"].items():
            if r is None:
                status = PANIC
                break
            if len(r["timer"]) == 0:
                status = INVALID
                break
            s = parse(r["timer"])
            if s is None:
                status = INVALID
                break
            scheds.append(s)
        if status == OK:
            if j["kind"] == 1:
                j["parallels"] = 1
            ids = [j["id"]] + [x for r in j["rules"].items() for x in
                               [r["id"]] + r["gids"].items() + r["nids"].items() + r["exclude_nids"].items()]
            if any(b"\x00" in x for x in ids):
                status = UNSUPPORTED
        j["schedules"] = scheds
        st.append(status)
        jobs.append(j if status == OK else None)
    last = {}
    for i, j in enumerate(jobs):
        if j is not None:
            last[j["id"]] = i
    out = []
    for i, j in enumerate(jobs):
        if j is None:
            continue
        if last[j["id"]] != i:
            st[i] = REPLACED
            continue
        out.append((i, j))
    return st, out


def ingest_groups(docs):
    st, groups = [], []
    for d in docs:
        ok, g = _unmarshal(d, lambda: {"id": b"", "name": b"", "nids": GoSlice()}, GROUP_FIELDS,
                           lambda g, f, v: g.__setitem__(f, _strings(v, g[f]) if f == "nids"
                                                          else _store_string(v, g[f])))
        if ok and (b"\x00" in g["id"] or any(b"\x00" in x for x in g["nids"].items())):
            st.append(UNSUPPORTED)
            groups.append(None)
            continue
        st.append(OK if ok else UNMARSHAL)
        groups.append(g if ok else None)
    last = {}
    for i, g in enumerate(groups):
        if g is not None:
            last[g["id"]] = i
    out = []
    for i, g in enumerate(groups):
        if g is None:
            continue
        if last[g["id"]] != i:
            st[i] = REPLACED
            continue
        out.append((i, g))
    return st, out
