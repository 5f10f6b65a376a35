"""The reference's node/cron API surface, backed by the MI355X engine.

Mirrors qlchan/cronsun node/cron:
  Parse / ParseStandard / NewParser(options).Parse   parser.go:66-183
  SpecSchedule{Second, Minute, Hour, Dom, Month, Dow} spec.go:7-9
  ConstantDelaySchedule{Delay}, Every(duration)       constantdelay.go:7-27
  Schedule.Next(t)                                    spec.go:55-145, constantdelay.go:25-27
  ParseOption constants Second ... Descriptor          parser.go:17-26

Parsing runs on the host (C++ in libcronsun_gpu.so); Next runs on the GPU
through cg_next_batch.  Times are int unix seconds; Go's zero time.Time{} is
ZERO_TIME.  Parse errors raise ParseError carrying Go's message.
"""
import ctypes as C
import os

import numpy as np

from . import _lib
from ._lib import ZERO_TIME, check, lib

# ParseOption (parser.go:17-26)
Second = _lib.PARSE_SECOND
Minute = _lib.PARSE_MINUTE
Hour = _lib.PARSE_HOUR
Dom = _lib.PARSE_DOM
Month = _lib.PARSE_MONTH
Dow = _lib.PARSE_DOW
DowOptional = _lib.PARSE_DOW_OPTIONAL
Descriptor = _lib.PARSE_DESCRIPTOR

STAR_BIT = 1 << 63

NANOSECOND = 1
MICROSECOND = 1000
MILLISECOND = 1000 * MICROSECOND
SECOND_NS = 1000 * MILLISECOND
MINUTE_NS = 60 * SECOND_NS
HOUR_NS = 60 * MINUTE_NS


class ParseError(ValueError):
    """A spec the reference parser rejects (the Go error text is the message)."""


class GoPanic(ValueError):
    """An input on which the reference Go code panics (e.g. Parse("") indexes spec[0])."""


class Schedule:
    """cron.Schedule (cron.go:36-40)."""

    def Next(self, t, loc=None):
        from .engine import default_engine
        return int(default_engine().next_batch([self], loc, np.array([t], dtype=np.int64))[0])

    def to_c(self):
        raise NotImplementedError


class SpecSchedule(Schedule):
    __slots__ = ("Second", "Minute", "Hour", "Dom", "Month", "Dow")

    def __init__(self, Second=0, Minute=0, Hour=0, Dom=0, Month=0, Dow=0):
        self.Second, self.Minute, self.Hour = Second, Minute, Hour
        self.Dom, self.Month, self.Dow = Dom, Month, Dow

    def __eq__(self, o):
        return isinstance(o, SpecSchedule) and all(
            getattr(self, f) == getattr(o, f) for f in self.__slots__)

    def __repr__(self):
        return "&SpecSchedule{%s}" % ", ".join(f"{f}:{getattr(self, f):#x}" for f in self.__slots__)

    def to_c(self):
        s = _lib.cg_schedule()
        s.kind = 0
        s.second, s.minute, s.hour = self.Second, self.Minute, self.Hour
        s.dom, s.month, s.dow = self.Dom, self.Month, self.Dow
        return s


class ConstantDelaySchedule(Schedule):
    __slots__ = ("Delay",)

    def __init__(self, Delay):
        self.Delay = int(Delay)  # time.Duration, nanoseconds

    def __eq__(self, o):
        return isinstance(o, ConstantDelaySchedule) and o.Delay == self.Delay

    def __repr__(self):
        return f"ConstantDelaySchedule{{Delay:{self.Delay}}}"

    def to_c(self):
        s = _lib.cg_schedule()
        s.kind = 1
        s.delay_ns = self.Delay
        return s


def Every(duration_ns):
    """Every(d) -- constantdelay.go:14-21 (sub-second rounds up to 1 s)."""
    return ConstantDelaySchedule(lib().cg_every(int(duration_ns)))


def _from_c(s):
    if s.kind == 1:
        return ConstantDelaySchedule(s.delay_ns)
    return SpecSchedule(s.second, s.minute, s.hour, s.dom, s.month, s.dow)


class Parser:
    """Parser{options} -- parser.go:47-136."""

    def __init__(self, options):
        self.options = options

    def Parse(self, spec):
        b = spec.encode() if isinstance(spec, str) else bytes(spec)
        out = _lib.cg_schedule()
        err = C.create_string_buffer(1024)
        rc = lib().cg_parse(self.options, b, len(b), C.byref(out), err, 1024)
        if rc == _lib.CG_EPANIC:
            raise GoPanic(err.value.decode(errors="replace"))
        if rc != 0:
            raise ParseError(err.value.decode(errors="replace"))
        return _from_c(out)


def NewParser(options):
    return Parser(options)


_default = Parser(_lib.PARSE_DEFAULT)
_standard = Parser(_lib.PARSE_STANDARD)


def Parse(spec):
    """cron.Parse -- seconds-first 5/6-field specs and descriptors (parser.go:171-183)."""
    return _default.Parse(spec)


def ParseStandard(spec):
    """cron.ParseStandard -- 5-field minute-first specs (parser.go:155-169)."""
    return _standard.Parse(spec)


def parse_batch(specs, options=_lib.PARSE_DEFAULT, threads=8):
    """Multithreaded host parse of many specs -> (cg_schedule array, status int32 array)."""
    n = len(specs)
    enc = [s.encode() if isinstance(s, str) else bytes(s) for s in specs]
    bufs = (C.c_char_p * max(n, 1))(*enc) if n else (C.c_char_p * 1)()
    lens = np.array([len(b) for b in enc], dtype=np.uint64)
    out = (_lib.cg_schedule * max(n, 1))()
    status = np.zeros(max(n, 1), dtype=np.int32)
    check(lib().cg_parse_batch(options, C.cast(bufs, C.c_void_p), lens.ctypes.data, n,
                               C.cast(out, C.c_void_p), status.ctypes.data, threads))
    return out, status[:n]


def ParseDuration(s):
    """time.ParseDuration (used by "@every", parser.go:368-373); returns ns."""
    b = s.encode()
    v = C.c_int64()
    rc = lib().cg_parse_duration(b, len(b), C.byref(v))
    if rc != 0:
        raise ParseError(_lib.last_error())
    return v.value


# ---------------------------------------------------------------- locations
class Location:
    """A time zone (Go *time.Location), host-side rules handed to kernels."""

    def __init__(self, handle, name):
        self._h = handle
        self.name = name

    def __del__(self):
        try:
            if self._h:
                lib().cg_zone_free(self._h)
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def offset(self, t):
        o = C.c_int32()
        check(lib().cg_zone_offset(self._h, int(t), C.byref(o)))
        return o.value

    def __repr__(self):
        return f"Location({self.name})"


def _zoneinfo_dirs():
    dirs = []
    if os.environ.get("ZONEINFO"):
        dirs.append(os.environ["ZONEINFO"])
    try:
        import importlib.util
        spec = importlib.util.find_spec("tzdata")
        if spec and spec.origin:
            dirs.append(os.path.join(os.path.dirname(spec.origin), "zoneinfo"))
    except Exception:
        pass
    dirs += ["/usr/share/zoneinfo", "/usr/lib/go/lib/time/zoneinfo"]
    return dirs


def LoadLocationFromTZData(name, data):
    h = C.c_void_p()
    check(lib().cg_zone_from_tzif(data, len(data), C.byref(h)))
    return Location(h, name)


def LoadLocation(name):
    """time.LoadLocation: "UTC"/"" -> UTC, else a TZif file from $ZONEINFO,
    the tzdata package or /usr/share/zoneinfo."""
    if name in ("", "UTC"):
        return UTC()
    for d in _zoneinfo_dirs():
        p = os.path.join(d, name)
        if os.path.isfile(p):
            with open(p, "rb") as f:
                return LoadLocationFromTZData(name, f.read())
    raise FileNotFoundError(f"unknown time zone {name}")


def FixedZone(name, offset):
    h = C.c_void_p()
    check(lib().cg_zone_fixed(int(offset), C.byref(h)))
    return Location(h, name)


_utc = None


def UTC():
    global _utc
    if _utc is None:
        h = C.c_void_p()
        check(lib().cg_zone_utc(C.byref(h)))
        _utc = Location(h, "UTC")
    return _utc
