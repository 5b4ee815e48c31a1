"""Nested-class configuration objects (API of humanoid/envs/base/base_config.py:34-56).

A config is a class whose attributes may themselves be classes; instantiating the outer class
instantiates every nested class recursively, so ``cfg.env.num_envs`` works on the instance and
subclasses can override single fields.
"""
import inspect


class BaseConfig:
    def __init__(self) -> None:
        self.init_member_classes(self)

    @staticmethod
    def init_member_classes(obj):
        for name in dir(obj):
            if name == "__class__":
                continue
            member = getattr(obj, name)
            if inspect.isclass(member):
                inst = member()
                setattr(obj, name, inst)
                BaseConfig.init_member_classes(inst)
