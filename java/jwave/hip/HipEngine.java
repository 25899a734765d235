package jwave.hip;

/**
 * Loads the JNI glue (jni/jwave_hip_jni.c), which links libjwave_hip.so, the MI355X engine.
 * Every drop-in class calls {@link #load()} from its static initialiser; a missing library is
 * an UnsatisfiedLinkError at class load, never a silent CPU fallback.
 */
public final class HipEngine {
  private static volatile boolean loaded;

  private HipEngine() {}

  public static void load() {
    if (!loaded) {
      synchronized (HipEngine.class) {
        if (!loaded) {
          System.loadLibrary("jwave_hip_jni");
          loaded = true;
        }
      }
    }
  }

  /** Engine version string (jw_version). */
  public static String version() {
    load();
    return nVersion();
  }

  /**
   * Makes {@code ordinal} the calling thread's GPU (jw_set_device).  Transforms constructed with
   * a device ordinal call this before each native call, so a ForkJoin fan-out (the pattern of
   * ParallelTransform.java:83-86) can spread work over the node's GPUs.
   *
   * @throws IllegalArgumentException for a negative or out-of-range ordinal
   */
  public static void setDevice(int ordinal) {
    load();
    nSetDevice(ordinal);
  }

  /** Number of visible HIP devices (0 if none). */
  public static int deviceCount() {
    load();
    return nDeviceCount();
  }

  /**
   * Frees every device table the engine caches (FFT twiddles, chirp-z tables, MODWT filter
   * spectra): the device side of MODWTTransform.clearFilterCache (MODWTTransform.java:556).
   * Safe while other threads run transforms (they finish first); returns the bytes freed.
   */
  public static long releaseCaches() {
    load();
    return nReleaseCaches();
  }

  private static native String nVersion();
  private static native void nSetDevice(int ordinal);
  private static native int nDeviceCount();
  private static native long nReleaseCaches();
}
