"""Device runtime: streams (teacher/student overlap), hipGraph step capture."""
