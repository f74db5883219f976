"""Experiment flags (code/infras/exp_config.py:1-55): equation, kernel, nepoch (+ device)."""


class Config(object):

    def parse(self, kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)
        print("=================================")
        print("*", self.config_name)
        print("---------------------------------")
        for k, v in self.__class__.__dict__.items():
            if not k.startswith("_"):
                print("-", k, ":", getattr(self, k))
        print("=================================")

    def __str__(self):
        buff = "=================================\n*" + self.config_name + "\n"
        buff += "---------------------------------\n"
        for k, v in self.__class__.__dict__.items():
            if not k.startswith("_"):
                buff += "-" + str(k) + ":" + str(getattr(self, k)) + "\n"
        return buff + "=================================\n"


class ExpConfig(Config):
    equation = None
    kernel = None
    nepoch = 1000000
    device = None   # HIP device ordinal (added; the reference ran wherever JAX placed it)

    def __init__(self):
        super(ExpConfig, self).__init__()
        self.config_name = "Exp Config"
