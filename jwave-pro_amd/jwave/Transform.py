"""jwave.Transform -- the facade (src/main/java/jwave/Transform.java:43-512).

Every method catches ``JWaveException``, prints it and returns ``None``
(Transform.java:81-90); unchecked exceptions (IllegalArgumentException) propagate.
"""
import traceback

from .exceptions import JWaveException, JWaveFailure


class Transform:
    def __init__(self, transform, *args):
        if transform is None:
            raise JWaveFailure("Transform - given object is null!")
        self._transform = transform

    def getBasicTransform(self):
        return self._transform

    def _guard(self, fn, *a):
        try:
            return fn(*a)
        except JWaveException as e:
            e.showMessage()
            traceback.print_exc()
            return None

    def forward(self, arr, *levels):
        return self._guard(self._transform.forward, arr, *levels)

    def reverse(self, arr, *levels):
        return self._guard(self._transform.reverse, arr, *levels)

    def decompose(self, arr):
        return self._guard(self._transform.decompose, arr)

    def recompose(self, mat, *level):
        return self._guard(self._transform.recompose, mat, *level)
