"""String enums with case/dash-insensitive parsing (parity: reference ``utilities/enums.py:20-154``)."""
from enum import Enum
from typing import List, Optional, Type, TypeVar

_E = TypeVar("_E", bound="EnumStr")


class EnumStr(str, Enum):
    """``str``-valued enum whose members compare equal to their (case-insensitive) value."""

    @staticmethod
    def _name() -> str:
        return "Task"

    @classmethod
    def _allowed_matches(cls, source: str) -> List[str]:
        keys = [m.lower() for m in cls._member_names_]
        vals = [str(m.value).lower() for m in cls]
        if source == "key":
            return keys
        if source == "value":
            return vals
        return sorted(set(keys + vals))

    @classmethod
    def from_str(cls: Type[_E], value: str, source: str = "key") -> _E:
        norm = str(value).replace("-", "_").lower()
        for member in cls:
            key_ok = source in ("key", "any") and member.name.lower() == norm
            val_ok = source in ("value", "any") and str(member.value).replace("-", "_").lower() == norm
            if key_ok or val_ok:
                return member
        raise ValueError(f"Invalid {cls._name()}: expected one of {cls._allowed_matches(source)}, but got {value}.")

    def __eq__(self, other: object) -> bool:
        if isinstance(other, Enum):
            other = other.value
        if other is None or self.value is None:
            return other is None and self.value is None
        return str(self.value).lower() == str(other).lower()

    def __hash__(self) -> int:
        return hash(str(self.value).lower() if self.value is not None else None)

    def __str__(self) -> str:
        return str(self.value)


class DataType(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Data type"

    BINARY = "binary"
    MULTILABEL = "multi-label"
    MULTICLASS = "multi-class"
    MULTIDIM_MULTICLASS = "multi-dim multi-class"


class AverageMethod(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Average method"

    MICRO = "micro"
    MACRO = "macro"
    WEIGHTED = "weighted"
    NONE = None
    SAMPLES = "samples"


class MDMCAverageMethod(EnumStr):
    @staticmethod
    def _name() -> str:
        return "MDMC Average method"

    GLOBAL = "global"
    SAMPLEWISE = "samplewise"


class ClassificationTask(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Classification"

    BINARY = "binary"
    MULTICLASS = "multiclass"
    MULTILABEL = "multilabel"


class ClassificationTaskNoBinary(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Classification"

    MULTILABEL = "multilabel"
    MULTICLASS = "multiclass"


class ClassificationTaskNoMultilabel(EnumStr):
    @staticmethod
    def _name() -> str:
        return "Classification"

    BINARY = "binary"
    MULTICLASS = "multiclass"


def _maybe(value: Optional[str]) -> Optional[str]:
    return None if value is None else str(value)
