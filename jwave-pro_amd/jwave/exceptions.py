"""Exception classes of the reference (src/main/java/jwave/exceptions/).

``JWaveException`` is checked in Java (``extends Throwable``, JWaveException.java:32);
``JWaveFailure`` / ``JWaveError`` derive from it.  ``IllegalArgumentException`` is the
unchecked ``java.lang`` exception ``MODWTTransform.forwardMODWT`` throws (:257-282).
"""


class JWaveException(Exception):
    """jwave.exceptions.JWaveException"""

    def showMessage(self):
        print(f"JWave{self.__class__.__name__[5:]}: {self}")


class JWaveFailure(JWaveException):
    """jwave.exceptions.JWaveFailure"""


class JWaveError(JWaveException):
    """jwave.exceptions.JWaveError"""


class IllegalArgumentException(ValueError):
    """java.lang.IllegalArgumentException"""
