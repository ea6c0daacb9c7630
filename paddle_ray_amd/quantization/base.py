"""Quanter / observer base classes and the factory protocol (parity:
python/paddle/quantization/{base_quanter,base_observer,factory,wrapper}.py)."""
import abc
import functools

from ..nn.layer.layers import Layer


class BaseQuanter(Layer, metaclass=abc.ABCMeta):
    """A layer that simulates quantization of its input and exposes its parameters."""

    @abc.abstractmethod
    def forward(self, input):
        ...

    @abc.abstractmethod
    def scales(self):
        ...

    @abc.abstractmethod
    def zero_points(self):
        ...

    @abc.abstractmethod
    def quant_axis(self):
        ...

    @abc.abstractmethod
    def bit_length(self):
        ...


class BaseObserver(BaseQuanter, metaclass=abc.ABCMeta):
    """A quanter that only observes (returns its input) and computes thresholds."""

    @abc.abstractmethod
    def cal_thresholds(self):
        ...


class ClassWithArguments(metaclass=abc.ABCMeta):
    def __init__(self, *args, **kwargs):
        self._args, self._kwargs = args, kwargs

    @property
    def args(self):
        return self._args

    @property
    def kwargs(self):
        return self._kwargs

    @abc.abstractmethod
    def _get_class(self):
        ...

    def __str__(self):
        a = ",".join([str(x) for x in self.args] + [f"{k}={v}" for k, v in self.kwargs.items()])
        return f"{self.__class__.__name__}({a})"

    __repr__ = __str__


class QuanterFactory(ClassWithArguments):
    """Holds a quanter class and its construction arguments; ``_instance(layer)`` builds one
    quanter per quantized layer."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.partial_class = None

    def _instance(self, layer):
        if self.partial_class is None:
            self.partial_class = functools.partial(self._get_class(), *self.args, **self.kwargs)
        return self.partial_class(layer)


ObserverFactory = QuanterFactory


def quanter(class_name):
    """Decorator declaring a factory class ``class_name`` (in the caller's module) for a
    customized BaseQuanter subclass."""
    import inspect

    def wrapper(target_class):
        def init(self, *args, **kwargs):
            QuanterFactory.__init__(self, *args, **kwargs)

        factory = type(class_name, (QuanterFactory,),
                       {'__init__': init, '_get_class': lambda self: target_class})
        mod = inspect.getmodule(inspect.stack()[1][0])
        if mod is not None:
            setattr(mod, class_name, factory)
            if '__all__' in mod.__dict__:
                mod.__all__.append(class_name)
        return target_class
    return wrapper


class ObserveWrapper(Layer):
    """Runs an observer before (``observe_input``) or after the observed layer."""

    def __init__(self, observer, observed, observe_input=True):
        super().__init__()
        self._observer = observer
        self._observed = observed
        self._observe_input = observe_input

    def forward(self, *inputs, **kwargs):
        if self._observe_input:
            return self._observed(self._observer(*inputs, **kwargs), **kwargs)
        return self._observer(self._observed(*inputs, **kwargs), **kwargs)
