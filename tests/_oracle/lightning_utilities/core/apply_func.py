import dataclasses
from collections import OrderedDict, defaultdict
from typing import Any, Callable


def apply_to_collection(data: Any, dtype: Any, function: Callable, *args: Any, wrong_dtype: Any = None,
                        include_none: bool = True, **kwargs: Any) -> Any:
    if isinstance(data, dtype) and (wrong_dtype is None or not isinstance(data, wrong_dtype)):
        return function(data, *args, **kwargs)
    if isinstance(data, (dict, OrderedDict, defaultdict)):
        out = [(k, apply_to_collection(v, dtype, function, *args, wrong_dtype=wrong_dtype,
                                       include_none=include_none, **kwargs)) for k, v in data.items()]
        if isinstance(data, defaultdict):
            return type(data)(data.default_factory, OrderedDict(out))
        return type(data)(out)
    is_namedtuple = isinstance(data, tuple) and hasattr(data, "_fields")
    if isinstance(data, (list, tuple)):
        out = [apply_to_collection(d, dtype, function, *args, wrong_dtype=wrong_dtype,
                                   include_none=include_none, **kwargs) for d in data]
        return type(data)(*out) if is_namedtuple else type(data)(out)
    if dataclasses.is_dataclass(data) and not isinstance(data, type):
        return data
    return data
