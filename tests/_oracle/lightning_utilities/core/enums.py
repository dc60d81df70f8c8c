from enum import Enum
from typing import Optional


class StrEnum(str, Enum):
    @classmethod
    def from_str(cls, value: str, source: str = "key") -> Optional["StrEnum"]:
        for st in cls:
            if st.value.lower() == value.lower() or st.name.lower() == value.lower():
                return st
        return None

    def __eq__(self, other: object) -> bool:
        other = other.value if isinstance(other, Enum) else str(other)
        return self.value.lower() == other.lower()

    def __hash__(self) -> int:
        return hash(self.value.lower())
