"""Object protocol (reference: mgs/obj/base.py:22-35)."""
from abc import ABC, abstractmethod
from typing import Any, Dict, Tuple


class CollisionMeshObject(ABC):
    """An object with a collision mesh (.obj) used by candidate generation."""

    name: str
    object_id: str

    @property
    @abstractmethod
    def obj_file_path(self) -> str:
        ...

    @abstractmethod
    def to_xml(self) -> Tuple[str, Dict[str, Any]]:
        ...
