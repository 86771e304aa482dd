"""Base config helpers (reference: dll/configs/base_config.py:11-64)."""
import os
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, Optional

import yaml


@dataclass
class DeviceConfig:
    type: str = "auto"
    force_cpu: bool = False
    mixed_precision: bool = True
    pin_memory: bool = True


@dataclass
class BaseConfig:
    @classmethod
    def get_config_path(cls) -> str:
        """``$DLL_CONFIG_PATH`` or ``<project root>/configs/default_config.yaml``."""
        env = os.getenv("DLL_CONFIG_PATH")
        if env:
            return env
        here = Path(__file__).resolve().parent
        while here.name and not (here / "setup.py").exists():
            here = here.parent
        return str(here / "configs" / "default_config.yaml")

    def to_dict(self) -> Dict:
        return dict(self.__dict__)

    @classmethod
    def from_dict(cls, d: Dict) -> "BaseConfig":
        return cls(**d)

    @classmethod
    def from_default(cls, key: Optional[str] = None) -> "BaseConfig":
        with open(cls.get_config_path()) as f:
            d = yaml.safe_load(f)
        if key:
            for part in key.split("."):
                d = d[part]
        return cls.from_dict(d)

    def save_yaml(self, path: str) -> None:
        with open(path, "w") as f:
            yaml.safe_dump(self.to_dict(), f)

    def validate(self) -> None:
        pass
