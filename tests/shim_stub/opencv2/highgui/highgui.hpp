#include "../cv_stub.hpp"
