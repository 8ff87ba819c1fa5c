"""Minimal mirror of Kernel's expression API for scan filters
(kernel-api/src/main/java/io/delta/kernel/expressions/: Column.java, Literal.java, Predicate.java,
And.java, Or.java, AlwaysTrue.java). Names and argument meaning follow the reference so a filter
reads the same: ``Predicate(">", Column("id"), Literal.ofLong(25_000_000))``."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Column:
    names: tuple

    def __init__(self, *names):
        if len(names) == 1 and isinstance(names[0], (list, tuple)):
            names = tuple(names[0])
        object.__setattr__(self, "names", tuple(names))

    def __repr__(self):
        return "column(%s)" % ".".join("`%s`" % n for n in self.names)


@dataclass(frozen=True)
class Literal:
    value: object
    type: str            # Kernel DataType name: "long", "integer", "short", "byte", "string", ...

    @staticmethod
    def ofLong(v):
        return Literal(int(v), "long")

    @staticmethod
    def ofInt(v):
        return Literal(int(v), "integer")

    @staticmethod
    def ofShort(v):
        return Literal(int(v), "short")

    @staticmethod
    def ofByte(v):
        return Literal(int(v), "byte")

    @staticmethod
    def ofDate(days_since_epoch):                      # Literal.ofDate(int daysSinceEpochUTC)
        return Literal(int(days_since_epoch), "date")

    @staticmethod
    def ofTimestamp(micros_since_epoch_utc):             # Literal.ofTimestamp(long)
        return Literal(int(micros_since_epoch_utc), "timestamp")

    @staticmethod
    def ofDecimal(value, precision, scale):
        """Literal.ofDecimal(BigDecimal, int, int) (Literal.java:173-183): the value is stored with
        setScale(scale) (ArithmeticException when that needs rounding) and its precision must not
        exceed `precision`."""
        import decimal
        with decimal.localcontext() as ctx:
            ctx.prec = 200
            d = decimal.Decimal(value)
            q = d.quantize(decimal.Decimal(1).scaleb(-scale))
            if q != d:
                raise ArithmeticError("Rounding necessary")
            digits = len(q.as_tuple().digits)
            if digits > precision:
                raise ValueError("Decimal precision=%d for decimal %s exceeds max precision %d" % (digits, q, precision))
        return Literal(q, "decimal(%d,%d)" % (precision, scale))

    @staticmethod
    def ofTimestampNtz(micros):                          # Literal.ofTimestampNtz(long)
        return Literal(int(micros), "timestamp_ntz")

    @staticmethod
    def ofFloat(v):                                      # Literal.ofFloat(float): a binary32 value
        import struct
        return Literal(struct.unpack("<f", struct.pack("<f", float(v)))[0], "float")

    @staticmethod
    def ofDouble(v):
        return Literal(float(v), "double")

    @staticmethod
    def ofString(v):
        return Literal(str(v), "string")

    @staticmethod
    def ofBoolean(v):
        return Literal(bool(v), "boolean")

    @staticmethod
    def ofNull(t):
        return Literal(None, t)


@dataclass(frozen=True)
class Predicate:
    name: str
    children: tuple

    def __init__(self, name, *children):
        if len(children) == 1 and isinstance(children[0], (list, tuple)):
            children = tuple(children[0])
        object.__setattr__(self, "name", name)
        object.__setattr__(self, "children", tuple(children))


def And(left, right):
    return Predicate("AND", left, right)


def Or(left, right):
    return Predicate("OR", left, right)


ALWAYS_TRUE = Predicate("ALWAYS_TRUE")
