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

  private static native String nVersion();
}
