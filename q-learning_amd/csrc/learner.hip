// placeholder, replaced by the learner
#include "objects.h"
